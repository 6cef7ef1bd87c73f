#!/bin/bash
# attention backward v1 (128 keys/WG) vs v2 (256 keys/WG): numerics, microbench, end-to-end
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "attention or gpt2 or trainer" > gpurun_out/pytest_attn.log 2>&1 || { tail -40 gpurun_out/pytest_attn.log; exit 1; }
tail -1 gpurun_out/pytest_attn.log
for v in v1 v2 v1 v2; do
  ORION_ATTN_BWD=$v timeout -k 10 120 python scripts/bench_attn.py --B 64 --T 1024 --H 12 --D 64 > gpurun_out/attn_$v.log 2>&1 || { tail -20 gpurun_out/attn_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/attn_$v.log | cut -c1-200)"
done
for v in v1 v2; do
  ORION_ATTN_BWD=$v timeout -k 10 300 python bench.py > gpurun_out/bench_$v.log 2>&1 || { tail -20 gpurun_out/bench_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/bench_$v.log | cut -c1-160)"
done
