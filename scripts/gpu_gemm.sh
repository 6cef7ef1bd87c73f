#!/bin/bash
# csrc/gemm.hip: GPU tests, then the microbench (vs hipBLASLt) with output checks.
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-gemm}
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1 || { tail -60 gpurun_out/pytest_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_$TAG.log
timeout -k 10 300 python scripts/bench_gemm.py --check > gpurun_out/gemm_$TAG.log 2>&1
rc=$?; cat gpurun_out/gemm_$TAG.log | grep -v amdgpu.ids; exit $rc
