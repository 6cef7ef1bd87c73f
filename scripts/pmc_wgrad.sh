#!/bin/bash
# PMC counters for the wgrad kernel (kernel-trace only; counters in their own runs).
set -o pipefail
cd "$(dirname "$0")/.."
REPO=$(pwd)
mkdir -p gpurun_out/pmcw
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp
run() {
  tag=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $REPO/gpurun_out/pmcw -o $tag -- python3 $REPO/scripts/wgrad_one.py > $REPO/gpurun_out/pmcw/$tag.log 2>&1
}
run w1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT && \
run w2 SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC && \
run w3 SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL GRBM_GUI_ACTIVE && \
run w4 TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum SQ_INSTS_FLAT_LDS_ONLY
rc=$?
cd $REPO
for f in gpurun_out/pmcw/*counter_collection.csv; do
  python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(float); n = collections.Counter()
for r in rows:
    if "wgrad" not in r.get("Kernel_Name", ""):
        continue
    agg[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
print(sys.argv[1].split("/")[-1], {k: round(v / max(1, n[k]), 1) for k, v in agg.items()})
PY
done
exit $rc
