#!/bin/bash
# Same-box comparison of several extension builds: runs "$@" against every variants/_C_*.so
# in turn, ROUNDS rounds (default 2); prints the last output line of each run and keeps each
# run's log as gpurun_out/abv_<AB_TAG>_<variant>_r<round>.log.
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for r in $(seq ${ROUNDS:-2}); do
  for so in variants/_C_*.so; do
    v=$(basename $so .so)
    log=gpurun_out/abv_${AB_TAG:-x}_${v}_r$r.log
    ORION_AMD_EXT=$PWD/$so timeout -k 10 ${AB_TIMEOUT:-300} "$@" > $log 2>&1 || { echo "FAIL $v"; tail -20 $log; exit 1; }
    echo "$v $(tail -1 $log)"
  done
done
