#!/bin/bash
# Attention timing + per-kernel trace (+ optional PMC passes) on the GPT-2 and Llama-7B shapes.
# usage: scripts/attn_study.sh TAG [pmc]
set -o pipefail
cd "$(dirname "$0")/.."
REPO=$(pwd)
TAG=$1
OUT=$REPO/gpurun_out/attn_$TAG
mkdir -p $OUT
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
[ "$3" = skipbench ] || { timeout -k 10 180 python3 scripts/bench_attn.py --B 64 --T 1024 --H 12 --D 64 > $OUT/bench_gpt2.json 2> $OUT/bench_gpt2.err && \
timeout -k 10 180 python3 scripts/bench_attn.py --B 4 --T 4096 --H 32 --D 128 > $OUT/bench_llama.json 2> $OUT/bench_llama.err && \
cat $OUT/bench_gpt2.json $OUT/bench_llama.json; } && \
(cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tr_gpt2 -o t -- python3 $REPO/scripts/attn_one.py 64 1024 12 12 64 5 > $OUT/tr_gpt2.log 2>&1) && \
(cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tr_llama -o t -- python3 $REPO/scripts/attn_one.py 4 4096 32 32 128 5 > $OUT/tr_llama.log 2>&1) && \
for d in tr_gpt2 tr_llama; do f=$(find $OUT/$d -name '*kernel_stats.csv' | head -1); echo "== $d"; python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print("%-60s %6s %10.1f us" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
done
rc=$?
if [ $rc = 0 ] && [ "$2" = pmc ]; then bash scripts/pmc_attn_split.sh $TAG 64 1024 12 12 64; rc=$?; fi
exit $rc
