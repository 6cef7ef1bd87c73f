#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for args in "--model gpt2-tiny --seq-len 256 --micro-batch 8" "--micro-batch 8" "--micro-batch 64"; do
  for g in "--no-tuned-gemms" "--hip-graph"; do
    timeout -k 10 300 python bench.py $args $g --steps 20 --warmup 5 > gpurun_out/bg.log 2>&1 || { echo "FAILED: $args $g"; tail -8 gpurun_out/bg.log; exit 1; }
    python - "$args $g" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/bg.log").read().strip().splitlines()[-1])
print(sys.argv[1], d["value"], d["ms_per_step"], "graph", d.get("hip_graph"), "loss", d["loss"])
PY
  done
done
