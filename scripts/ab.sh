#!/bin/bash
# Same-box A/B: run "$@" alternately against variants/_C_base.so and the in-tree
# orion_amd/_C.so, 3 rounds; prints the last line of each run.
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in base new; do
    if [[ $v == base ]]; then ext=$PWD/variants/_C_base.so; else ext=$PWD/orion_amd/_C.so; fi
    ORION_AMD_EXT=$ext timeout -k 10 ${AB_TIMEOUT:-300} "$@" > gpurun_out/ab_$v.log 2>&1 || { echo "FAIL $v"; tail -20 gpurun_out/ab_$v.log; exit 1; }
    echo "$v $(tail -1 gpurun_out/ab_$v.log)"
  done
done
