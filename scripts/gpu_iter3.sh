#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q -k "wgrad or slab" > gpurun_out/pytest_wgrad.log 2>&1 || { tail -60 gpurun_out/pytest_wgrad.log; exit 1; }
tail -1 gpurun_out/pytest_wgrad.log
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 600 python scripts/bench_gemms.py > gpurun_out/gemms_hip.log 2>&1 || { tail -20 gpurun_out/gemms_hip.log; exit 1; }
tail -1 gpurun_out/gemms_hip.log
ORION_WGRAD=bmm timeout -k 10 600 python scripts/bench_gemms.py > gpurun_out/gemms_bmm.log 2>&1 || { tail -20 gpurun_out/gemms_bmm.log; exit 1; }
tail -1 gpurun_out/gemms_bmm.log
AB_COLS=150 bash scripts/ab_repo.sh python bench.py --steps 10 --warmup 3 || exit 1
