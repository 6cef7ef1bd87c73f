#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q -k "hip_graph" > gpurun_out/pytest_graph.log 2>&1 || { tail -40 gpurun_out/pytest_graph.log; exit 1; }
tail -1 gpurun_out/pytest_graph.log
for args in "--micro-batch 64" "--micro-batch 8" "--model gpt2-tiny --seq-len 256 --micro-batch 8"; do
  for g in "--no-tuned-gemms" "--hip-graph"; do
    timeout -k 10 300 python bench.py $args $g --steps 20 --warmup 5 > gpurun_out/bg.log 2>&1 || { tail -30 gpurun_out/bg.log; exit 1; }
    python - "$args $g" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/bg.log").read().strip().splitlines()[-1])
print(sys.argv[1], d["value"], d["ms_per_step"], "graph", d.get("hip_graph"), "loss", d["loss"])
PY
  done
done
