#!/bin/bash
# PMC counters for the attention kernels (own run, kernel-trace only, no sys/runtime trace).
set -o pipefail
cd "$(dirname "$0")/.."
REPO=$(pwd)
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true
grep -o -E "SQ_[A-Z0-9_]+" gpurun_out/pmc/counters_list.txt | sort -u > gpurun_out/pmc/sq_counters.txt || true
cd /tmp
run() {  # $1 = tag, rest = counters
  tag=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $REPO/gpurun_out/pmc -o $tag -- python3 $REPO/scripts/bench_attn.py --iters 3 ${ATTN_ARGS:-} > $REPO/gpurun_out/pmc/$tag.log 2>&1
}
run p1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT && \
run p2 SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC && \
run p3 SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL GRBM_GUI_ACTIVE
rc=$?
cd $REPO
python3 scripts/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc/summary.txt 2>&1 && cat gpurun_out/pmc/summary.txt
ls gpurun_out/pmc | head -30
exit $rc
