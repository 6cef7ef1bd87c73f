#!/bin/bash
# A/B of the split-backward dK/dV kernel forms in one box: tests for the default form, then
# bench_attn at the GPT-2 and Llama-7B shapes under ORION_ATTN_KV=reg and =dma.
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-kvab}
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
for form in reg reg; do
  for shape in "--B 64 --T 1024 --H 12 --D 64" "--B 4 --T 4096 --H 32 --Hkv 8 --D 128 --iters 10"; do
    ORION_ATTN_KV=$form timeout -k 10 120 python scripts/bench_attn.py $shape 2>/dev/null | \
      python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('$form', r['D'], 'split', r['bwd_split_ms'], 'fwd', r['fwd_ms'])" || exit 1
  done
done
