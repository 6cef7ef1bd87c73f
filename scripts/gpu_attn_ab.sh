#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -m pytest tests/test_kernels_gpu.py -x -q -k "attention or gpt2 or llama" > gpurun_out/pytest_attn.log 2>&1 || { tail -60 gpurun_out/pytest_attn.log; exit 1; }
tail -1 gpurun_out/pytest_attn.log
bash scripts/ab.sh python scripts/bench_attn.py --B 64 ${ATTN_ARGS:-} || exit 1
