#!/bin/bash
# Steady-state kernel summary of the bench step under one environment:
#   scripts/prof_steady.sh TAG [VAR=value ...] [-- bench args]
# rocprofv3 kernel trace of bench.py (default --steps 3 --warmup 2), condensed by
# scripts/prof_summary.py --steady into gpurun_out/prof_TAG_steady.txt.
set -o pipefail
cd "$(dirname "$0")/.."
REPO=$(pwd)
TAG=$1; shift
while [ $# -gt 0 ] && [ "$1" != "--" ]; do export "$1"; shift; done
[ "$1" == "--" ] && shift
ARGS=${@:-"--steps 3 --warmup 2"}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
d=$REPO/gpurun_out/prof_$TAG; rm -rf $d; mkdir -p $d
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python3 $REPO/bench.py $ARGS > $d/bench.log 2>&1) || { tail -20 $d/bench.log; exit 1; }
f=$(find $d -name "*kernel_trace.csv" | head -1)
python3 scripts/prof_summary.py "$f" --steady > gpurun_out/prof_${TAG}_steady.txt
rm -f "$f"
head -45 gpurun_out/prof_${TAG}_steady.txt
