#!/bin/bash
# One GPU iteration: kernel tests, whole-tree A/B of the bench vs variants/base_repo
# (untuned GEMMs on both sides), then the tuned bench of this tree.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
AB_COLS=120 bash scripts/ab_repo.sh python bench.py --micro-batch 64 --grad-accum 1 --steps 10 --warmup 3 --no-tuned-gemms || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_tuned.log 2>&1 || { tail -20 gpurun_out/bench_tuned.log; exit 1; }
tail -1 gpurun_out/bench_tuned.log
