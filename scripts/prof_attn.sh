#!/bin/bash
# rocprofv3 kernel stats of the attention microbench (per-kernel average time per call).
# usage: scripts/prof_attn.sh TAG [bench_attn args...]
set -o pipefail
cd "$(dirname "$0")/.."
REPO=$(pwd)
TAG=$1; shift
mkdir -p gpurun_out/prof_$TAG
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
   -d $REPO/gpurun_out/prof_$TAG -o run -- python3 $REPO/scripts/bench_attn.py --iters 5 "$@" \
   > $REPO/gpurun_out/prof_$TAG/bench.log 2>&1) || { tail -20 gpurun_out/prof_$TAG/bench.log; exit 1; }
f=$(find gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -1)
python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    n = r["Name"]
    if "attn" in n:
        print(f'{n[:60]:60s} calls {r["Calls"]:>5s} avg {float(r["AverageNs"])/1e6:8.4f} ms')
PY
