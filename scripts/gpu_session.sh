#!/bin/bash
# One GPU-box validation session: GPU tests, the 1-GPU headline bench, and a rocprofv3
# kernel profile of a short bench run. Every GPU step has its own time limit and the
# chain stops at the first failure.  usage: scripts/gpu_session.sh TAG [test|bench|prof|all]
set -o pipefail
cd "$(dirname "$0")/.."
REPO=$(pwd)
TAG=${1:-r02}
STEP=${2:-all}
mkdir -p gpurun_out/prof_$TAG
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
if [[ $STEP == all || $STEP == test ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
    > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
  tail -3 gpurun_out/pytest_gpu_$TAG.log
fi
if [[ $STEP == all || $STEP == bench ]]; then
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$TAG.log 2>&1 \
    || { tail -40 gpurun_out/bench_$TAG.log; exit 1; }
  tail -1 gpurun_out/bench_$TAG.log
fi
if [[ $STEP == all || $STEP == prof ]]; then
  # profile covers warmup + steps = 5 steps
  (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
     -d $REPO/gpurun_out/prof_$TAG -o run -- python3 $REPO/bench.py --steps 3 --warmup 2 \
     > $REPO/gpurun_out/prof_$TAG/bench.log 2>&1) || { tail -30 gpurun_out/prof_$TAG/bench.log; exit 1; }
  f=$(find gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -1)
  python scripts/prof_summary.py "$f" --steps 5 > gpurun_out/prof_$TAG/summary.txt && head -40 gpurun_out/prof_$TAG/summary.txt
fi
