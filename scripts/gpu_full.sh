#!/bin/bash
# tests -> bench (native) -> rocprofv3 profile; stops at the first failing step.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench_native.log 2>&1 || { tail -40 gpurun_out/bench_native.log; exit 1; }
tail -1 gpurun_out/bench_native.log
timeout -k 10 300 python scripts/bench_attn.py > gpurun_out/bench_attn.log 2>&1 && tail -1 gpurun_out/bench_attn.log
if [[ -z "$NOPROF" ]]; then bash scripts/profile.sh --steps 3 --warmup 2 > /dev/null 2>&1; echo "profile rc=$?"; fi
