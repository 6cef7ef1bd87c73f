#!/bin/bash
# rocprofv3 kernel trace + stats of a short bench run; summaries land in gpurun_out/prof.
set -o pipefail
cd "$(dirname "$0")/.."
REPO=$(pwd)
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
export HSA_ENABLE_IPC_MODE_LEGACY=0
ARGS=${@:-"--steps 3 --warmup 2"}  # NOTE: the profile covers warmup + steps; divide by their sum
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $REPO/gpurun_out/prof -o run -- python3 $REPO/bench.py $ARGS > $REPO/gpurun_out/prof/bench.log 2>&1
rc=$?
cd $REPO
find gpurun_out/prof -name "*kernel_stats.csv" | head -3
f=$(find gpurun_out/prof -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && head -40 "$f"
exit $rc
