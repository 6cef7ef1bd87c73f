#!/bin/bash
# PMC counter passes (kernel-trace only, each pass its own run) for one csrc/gemm16.hip shape.
# usage: scripts/pmc_gemm.sh TAG M N K wkm epi
set -o pipefail
cd "$(dirname "$0")/.."
REPO=$(pwd)
TAG=$1; shift
OUT=$REPO/gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp
run() {
  p=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $OUT -o $p \
    -- python3 $REPO/scripts/gemm_one.py $ARGS > $OUT/$p.log 2>&1
}
ARGS="$*"
run p1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT && \
run p2 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE && \
run p3 TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum && \
run p4 TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES GRBM_GUI_ACTIVE
rc=$?
cd $REPO
python3 scripts/pmc_summary.py $OUT
exit $rc
