#!/bin/bash
# micro-batch / grad-accum sweep at fixed 65536 tokens per step (untuned GEMMs for all, fair A/B)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for cfg in "32 2" "64 1" "16 4" "8 8"; do
  set -- $cfg
  timeout -k 10 240 python bench.py --micro-batch $1 --grad-accum $2 --steps 10 --warmup 3 --no-tuned-gemms > gpurun_out/sweep_$1_$2.log 2>&1 || { echo "fail $cfg"; tail -5 gpurun_out/sweep_$1_$2.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/sweep_$1_$2.log').read().strip().splitlines()[-1]); print('mb', $1, 'accum', $2, d['value'], d['ms_per_step'])"
done
