#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for cfg in 0 2 3 4; do
  ORION_WGRAD_CFG=$cfg timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q -k "wgrad_kernel or strided" > gpurun_out/pytest_wgrad_$cfg.log 2>&1 || { echo "cfg $cfg FAILED"; tail -40 gpurun_out/pytest_wgrad_$cfg.log; exit 1; }
  echo "cfg $cfg $(tail -1 gpurun_out/pytest_wgrad_$cfg.log)"
done
for cfg in 0 2 3 4 0 2; do
  ORION_WGRAD=hip ORION_WGRAD_CFG=$cfg timeout -k 10 600 python scripts/bench_gemms.py > gpurun_out/gemms_cfg$cfg.log 2>&1 || { tail -20 gpurun_out/gemms_cfg$cfg.log; exit 1; }
  python - "$cfg" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/gemms_cfg{sys.argv[1]}.log").read().strip().splitlines()[-1])
print("cfg", sys.argv[1], {k: (v["dw_ms"], v["dw_PF"]) for k, v in d.items() if isinstance(v, dict)}, "step", d["step_gemm_ms"])
PY
done
