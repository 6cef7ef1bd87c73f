#!/bin/bash
# bench_gemm.py under each ORION_GEMM_CFG given (after the GEMM tests).  usage: TAG CFG...
set -o pipefail
cd "$(dirname "$0")/.."
TAG=$1; shift
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for c in "$@"; do
  ORION_GEMM_CFG=$c timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/pytest_${TAG}_$c.log 2>&1 || { tail -30 gpurun_out/pytest_${TAG}_$c.log; exit 1; }
  ORION_GEMM_CFG=$c timeout -k 10 300 python scripts/bench_gemm.py > gpurun_out/gemm_${TAG}_$c.log 2>&1 || exit 1
  echo "cfg $c: $(tail -1 gpurun_out/gemm_${TAG}_$c.log)"
  python3 -c "
import json,sys
for l in open('gpurun_out/gemm_${TAG}_$c.log'):
    if l.startswith('{\"shape'):
        r=json.loads(l); print(f\"  {r['shape']:26s} hip {r['hip_TFs']:7.1f}  blas {r['blas_TFs']:7.1f}\")
"
done
