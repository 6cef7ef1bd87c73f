#!/bin/bash
# GPU tests + attention microbench + bench configs (same box, back to back).
# CFGS="64x1 96x1" selects micro-batch x grad-accum configs (default "32x2 64x1").
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
if [[ -z "${SKIP_TESTS:-}" ]]; then
  timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
  tail -1 gpurun_out/pytest_gpu.log
fi
timeout -k 10 300 python scripts/bench_attn.py > gpurun_out/bench_attn.log 2>&1 && tail -1 gpurun_out/bench_attn.log || exit 1
for cfg in ${CFGS:-32x2 64x1}; do
  mb=${cfg%x*}; ac=${cfg#*x}
  timeout -k 10 300 python bench.py --micro-batch $mb --grad-accum $ac --steps 10 --warmup 3 ${BENCH_ARGS:-} > gpurun_out/bench_${mb}_${ac}.log 2>&1 || { tail -20 gpurun_out/bench_${mb}_${ac}.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/bench_${mb}_${ac}.log').read().strip().splitlines()[-1]); print('mb', $mb, 'accum', $ac, d['value'], d['ms_per_step'], 'tuned', d.get('tuned_gemm_entries'))"
done
