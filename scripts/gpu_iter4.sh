#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
AB_COLS=150 bash scripts/ab_repo.sh python bench.py --steps 10 --warmup 3 || exit 1
bash scripts/pmc_attn.sh > gpurun_out/pmc_attn_run.log 2>&1 || { tail -20 gpurun_out/pmc_attn_run.log; exit 1; }
for f in gpurun_out/pmc/p*_counter_collection.csv; do
  python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
for kname in ("attn_fwd", "attn_bwd_kernel"):
    agg = collections.defaultdict(float); n = collections.Counter()
    for r in rows:
        if kname not in r.get("Kernel_Name", ""):
            continue
        agg[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    print(sys.argv[1].split("/")[-1], kname, {k: round(v / max(1, n[k]), 1) for k, v in agg.items()})
PY
done
