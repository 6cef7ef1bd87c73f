#!/bin/bash
# Attention: GPU tests of the backward forms, then the microbench at the GPT-2 and
# Llama-7B shapes.  usage: scripts/gpu_attn.sh TAG
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-attn}
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_attention_gpu.py -x -v --timeout 240 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1 || { tail -60 gpurun_out/pytest_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_$TAG.log
timeout -k 10 300 python scripts/bench_attn.py --B 64 --T 1024 --H 12 --D 64 > gpurun_out/attn_$TAG.log 2>&1 &&
timeout -k 10 300 python scripts/bench_attn.py --B 4 --T 4096 --H 32 --Hkv 8 --D 128 --iters 10 >> gpurun_out/attn_$TAG.log 2>&1
rc=$?; cat gpurun_out/attn_$TAG.log; exit $rc
