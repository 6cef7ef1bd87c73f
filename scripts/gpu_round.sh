#!/bin/bash
# One GPU-box session: kernel numerics tests, then benches. Each GPU step has its own
# time limit and the chain stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
STEP=${1:-all}
run() { echo "=== $*" ; "$@"; }
if [[ $STEP == all || $STEP == test ]]; then
  run timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -50 gpurun_out/pytest_gpu.log; exit 1; }
  tail -5 gpurun_out/pytest_gpu.log
fi
if [[ $STEP == all || $STEP == bench ]]; then
  run timeout -k 10 300 python bench.py --impl native --steps 10 --warmup 3 > gpurun_out/bench_native.log 2>&1 || { tail -40 gpurun_out/bench_native.log; exit 1; }
  tail -2 gpurun_out/bench_native.log
  run timeout -k 10 300 python bench.py --impl torch --steps 10 --warmup 3 > gpurun_out/bench_torch.log 2>&1 || { tail -40 gpurun_out/bench_torch.log; exit 1; }
  tail -2 gpurun_out/bench_torch.log
fi
