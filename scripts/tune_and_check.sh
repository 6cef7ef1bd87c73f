#!/bin/bash
# Tune GEMMs for the default bench shapes, then A/B untuned / committed table / fresh table on the same box.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash scripts/tune_gemms.sh --steps 2 --warmup 1 || exit 1
T=$(ls gpurun_out/tunableop/tunableop_results*.csv | head -1)
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-tuned-gemms > gpurun_out/ab_untuned.log 2>&1 || exit 1
  echo "untuned $(tail -1 gpurun_out/ab_untuned.log | cut -c1-200)"
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --gemm-table $T > gpurun_out/ab_tuned.log 2>&1 || exit 1
  echo "fresh   $(tail -1 gpurun_out/ab_tuned.log | cut -c1-200)"
done
