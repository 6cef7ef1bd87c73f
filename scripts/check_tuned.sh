#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
PYTORCH_TUNABLEOP_VERBOSE=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_tuned_verbose.log 2>&1 || { tail -30 gpurun_out/bench_tuned_verbose.log; exit 1; }
grep -i -E "tunable|reading|could not|validat" gpurun_out/bench_tuned_verbose.log | head -20
tail -1 gpurun_out/bench_tuned_verbose.log
bash scripts/profile.sh --steps 3 --warmup 2
