#!/bin/bash
# Llama-2-7B shape, seq 4096, on one MI355X (BASELINE config 4): full training steps.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for mb in ${LLAMA_MBS:-1 4}; do
  timeout -k 10 600 python bench.py --model llama2-7b --seq-len 4096 --micro-batch $mb --grad-accum 1 --steps 3 --warmup 2 > gpurun_out/llama7b_mb$mb.log 2>&1 || { tail -30 gpurun_out/llama7b_mb$mb.log; exit 1; }
  tail -1 gpurun_out/llama7b_mb$mb.log
done
