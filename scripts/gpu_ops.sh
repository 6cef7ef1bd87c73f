#!/bin/bash
# Memory-bound op A/B (base vs new build) + wgrad GEMM study (untuned and TunableOp-tuned).
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
bash scripts/ab.sh python scripts/bench_ops.py || exit 1
timeout -k 10 300 python scripts/bench_wgrad.py > gpurun_out/wgrad_untuned.log 2>&1 || { tail -20 gpurun_out/wgrad_untuned.log; exit 1; }
tail -1 gpurun_out/wgrad_untuned.log
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=40 \
  PYTORCH_TUNABLEOP_FILENAME=gpurun_out/wgrad_tune.csv timeout -k 10 600 python scripts/bench_wgrad.py > gpurun_out/wgrad_tuned.log 2>&1 || { tail -20 gpurun_out/wgrad_tuned.log; exit 1; }
tail -1 gpurun_out/wgrad_tuned.log
