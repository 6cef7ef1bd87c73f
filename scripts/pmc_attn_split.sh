#!/bin/bash
# PMC passes (kernel-trace only, one run per pass) for the attention kernels on one shape.
# usage: scripts/pmc_attn_split.sh TAG B T Hq Hkv D
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
    -- python3 $REPO/scripts/attn_one.py $ARGS > $OUT/$p.log 2>&1
}
ARGS="$*"
run p1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT && \
run p2 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE && \
run p3 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE
rc=$?
cd $REPO
python3 scripts/pmc_summary.py $OUT attn
exit $rc
