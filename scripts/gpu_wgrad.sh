#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q -k "wgrad or slab" > gpurun_out/pytest_wgrad.log 2>&1 || { tail -60 gpurun_out/pytest_wgrad.log; exit 1; }
tail -1 gpurun_out/pytest_wgrad.log
ORION_WGRAD=hip timeout -k 10 600 python scripts/bench_gemms.py > gpurun_out/gemms_hip.log 2>&1 || { tail -20 gpurun_out/gemms_hip.log; exit 1; }
tail -1 gpurun_out/gemms_hip.log
ORION_WGRAD=bmm timeout -k 10 600 python scripts/bench_gemms.py > gpurun_out/gemms_bmm.log 2>&1 || { tail -20 gpurun_out/gemms_bmm.log; exit 1; }
tail -1 gpurun_out/gemms_bmm.log
