#!/bin/bash
# Targeted GPU check: selected tests (-k EXPR) then the 1-GPU bench with extra args.
# usage: scripts/gpu_quick.sh TAG "PYTEST_K_EXPR" "BENCH ARGS" ["BENCH ARGS 2"]
set -o pipefail
cd "$(dirname "$0")/.."
TAG=$1; K=$2; shift 2
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
if [[ -n "$K" ]]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "$K" \
    > gpurun_out/pytest_$TAG.log 2>&1 || { tail -60 gpurun_out/pytest_$TAG.log; exit 1; }
  tail -3 gpurun_out/pytest_$TAG.log
fi
i=0
for args in "$@"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py $args > gpurun_out/bench_${TAG}_$i.log 2>&1 \
    || { tail -40 gpurun_out/bench_${TAG}_$i.log; exit 1; }
  echo "bench $i ($args):"; tail -1 gpurun_out/bench_${TAG}_$i.log
done
