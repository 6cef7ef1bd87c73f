#!/bin/bash
# GPU tests, then the GPT-2 headline bench and the Llama-7B seq-4096 bench (same box).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
if [[ -z "${SKIP_TESTS:-}" ]]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
  tail -1 gpurun_out/pytest_gpu.log
fi
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench_gpt2.log 2>&1 || { tail -20 gpurun_out/bench_gpt2.log; exit 1; }
tail -1 gpurun_out/bench_gpt2.log | cut -c1-220
if [[ -z "${SKIP_LLAMA:-}" ]]; then
  timeout -k 10 600 python bench.py --model llama2-7b --seq-len 4096 --micro-batch ${LLAMA_MB:-4} --steps 3 --warmup 2 > gpurun_out/bench_llama.log 2>&1 || { tail -20 gpurun_out/bench_llama.log; exit 1; }
  tail -1 gpurun_out/bench_llama.log | cut -c1-220
fi
