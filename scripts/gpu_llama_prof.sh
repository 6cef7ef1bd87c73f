#!/bin/bash
# rocprofv3 kernel stats of the Llama-2-7B-shape seq-4096 training step (BASELINE config 4).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
MB=${LLAMA_MB:-4}
rm -rf gpurun_out/prof
bash scripts/profile.sh --model llama2-7b --seq-len 4096 --micro-batch $MB --steps 2 --warmup 1 > gpurun_out/profile_llama.log 2>&1 || { tail -30 gpurun_out/profile_llama.log; exit 1; }
tail -1 gpurun_out/prof/bench.log | cut -c1-300
python scripts/prof_summary.py gpurun_out/prof/run_kernel_stats.csv --steps 3 --top 40 > gpurun_out/prof_llama_summary.txt
cat gpurun_out/prof_llama_summary.txt
