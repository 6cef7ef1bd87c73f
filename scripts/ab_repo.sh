#!/bin/bash
# Same-box A/B of whole trees: variants/base_repo (a `git archive` of the base commit with
# its own build) vs this tree; runs "$@" from each tree's root, 3 alternating rounds.
cd "$(dirname "$0")/.."
ROOT=$PWD
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in base new; do
    if [[ $v == base ]]; then dir=$ROOT/variants/base_repo; else dir=$ROOT; fi
    (cd $dir && timeout -k 10 ${AB_TIMEOUT:-300} "$@") > gpurun_out/abr_$v.log 2>&1 || { echo "FAIL $v"; tail -20 gpurun_out/abr_$v.log; exit 1; }
    echo "$v $(tail -1 gpurun_out/abr_$v.log | cut -c1-${AB_COLS:-400})"
  done
done
