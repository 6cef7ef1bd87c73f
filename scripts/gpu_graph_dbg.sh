#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for cfg in "--micro-batch 8" "--micro-batch 64"; do
  for g in "--no-tuned-gemms" "--hip-graph"; do
    ORION_GRAPH_MAX_TOKENS=1000000 ORION_BENCH_TRACE_LOSS=1 timeout -k 10 300 python bench.py $cfg $g --steps 10 --warmup 5 > gpurun_out/bg.log 2> gpurun_out/bg.err || { echo "FAIL $cfg $g"; tail -5 gpurun_out/bg.err; exit 1; }
    echo "$cfg $g: $(grep -o 'loss [0-9a-z.]*' gpurun_out/bg.err | sed 's/loss //' | tail -4 | tr '\n' ' ')"
    ORION_GRAPH_MAX_TOKENS=1000000 timeout -k 10 300 python bench.py $cfg $g --steps 20 --warmup 5 > gpurun_out/bg.log 2> gpurun_out/bg.err || { echo "FAIL $cfg $g"; tail -5 gpurun_out/bg.err; exit 1; }
    python - "$cfg $g" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/bg.log").read().strip().splitlines()[-1])
print("   untraced", sys.argv[1], d["value"], d["ms_per_step"], "graph", d.get("hip_graph"), "loss", d["loss"])
PY
  done
done
