#!/bin/bash
# Whole-training-step PMC passes (each its own rocprofv3 run with --kernel-trace only):
#   m: MFMA busy cycles, MFMA / VALU instruction counts, GPU-active cycles
#   f: HBM-side fetch bytes (TCC FETCH_SIZE)      w: write bytes (TCC WRITE_SIZE)
#   l (PMC_LDS=1): LDS bank conflicts / LDS-active cycles, LDS and any-dependency waits
# over a 2-step GPT-2 bench, then the per-kernel-group table of scripts/pmc_step_summary.py.
# usage: [PMC_PASS_TIMEOUT=seconds] [PMC_SKIP_STEPS=n] scripts/pmc_step.sh TAG [bench args]
# (PMC_SKIP_STEPS: leave the first n optimizer steps -- the bench's warmup -- out of the table)
set -o pipefail
cd "$(dirname "$0")/.."
REPO=$(pwd)
TAG=${1:-step}; shift
ARGS=${*:-"--steps 1 --warmup 1"}
OUT=$REPO/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp || exit 1
run() {
  p=$1; shift
  # shellcheck disable=SC2086
  timeout -s KILL "${PMC_PASS_TIMEOUT:-150}" rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "$OUT/$p" -o run \
    -- python3 "$REPO/bench.py" $ARGS > "$OUT/$p.log" 2>&1 || { tail -20 "$OUT/$p.log"; return 1; }
}
run m SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE && \
run f FETCH_SIZE GRBM_GUI_ACTIVE && \
run w WRITE_SIZE GRBM_GUI_ACTIVE && \
{ [[ -z $PMC_LDS ]] || run l SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE; }
rc=$?
cd "$REPO" || exit 1
python3 scripts/pmc_step_summary.py "$OUT" "${PMC_SKIP_STEPS:-0}" > "$OUT/summary.txt" && cat "$OUT/summary.txt"
exit $rc
