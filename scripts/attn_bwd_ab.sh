#!/bin/bash
# GPU attention tests on the current build, then a same-box A/B of variants/_C_*.so on the
# GPT-2 and Llama-7B attention shapes (scripts/attn_fwd_time.py: forward + split backward).
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/attn_tests.log 2>&1 || { tail -30 gpurun_out/attn_tests.log; exit 1; }
tail -1 gpurun_out/attn_tests.log
for r in 1 2 3; do
  for so in variants/_C_*.so; do
    ORION_AMD_EXT=$PWD/$so timeout -k 10 120 python scripts/attn_fwd_time.py 64 1024 12 12 64 || exit 1
    ORION_AMD_EXT=$PWD/$so timeout -k 10 120 python scripts/attn_fwd_time.py 4 4096 32 32 128 || exit 1
  done
done
