#!/bin/bash
# Kernel-trace profiles of the headline bench under several environment settings, one
# rocprofv3 run each (steady-state summaries via scripts/prof_summary.py --steady and per-shape
# GEMM rows via scripts/prof_shapes.py).  usage: scripts/prof_ab.sh TAG "ENV_A" ["ENV_B" ...]
set -o pipefail
cd "$(dirname "$0")/.."
REPO=$(pwd)
TAG=$1; shift
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
i=0
for e in "$@"; do
  d=$REPO/gpurun_out/prof_${TAG}_$i
  mkdir -p $d
  echo "$e" > $d/env.txt
  ( for kv in $e; do export "$kv"; done
    cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $d -o run \
      -- python3 $REPO/bench.py --steps 4 --warmup 2 > $d/bench.log 2>&1 ) || { tail -20 $d/bench.log; exit 1; }
  f=$(find $d -name "*kernel_trace.csv" | head -1)
  python scripts/prof_summary.py "$f" --steady > $d/summary.txt && python scripts/prof_shapes.py "$f" > $d/shapes.txt
  echo "== [$e]"; head -32 $d/summary.txt
  i=$((i+1))
done
