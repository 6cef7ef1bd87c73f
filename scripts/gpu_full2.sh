#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || { tail -20 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log | cut -c1-200
rm -rf gpurun_out/prof
bash scripts/profile.sh --steps 5 --warmup 3 > gpurun_out/profile_run.log 2>&1 || { tail -20 gpurun_out/profile_run.log; exit 1; }
python scripts/prof_summary.py gpurun_out/prof/run_kernel_stats.csv --steps 8 > gpurun_out/prof_summary.txt
head -25 gpurun_out/prof_summary.txt; tail -2 gpurun_out/prof_summary.txt
