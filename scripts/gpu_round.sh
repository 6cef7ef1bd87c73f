#!/bin/bash
# Headline + Llama measurements on one GPU box: GPT-2-124M bench, its rocprofv3 kernel
# summary, then the Llama-2-7B-shape seq-4096 bench and its kernel summary.
# usage: scripts/gpu_round.sh TAG [gpt2|llama|all]
set -o pipefail
cd "$(dirname "$0")/.."
REPO=$(pwd)
TAG=${1:-round}; WHAT=${2:-all}
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
prof() {  # prof NAME STEPS_TOTAL bench-args...
  name=$1; tot=$2; shift 2
  mkdir -p gpurun_out/prof_${TAG}_$name
  (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
     -d $REPO/gpurun_out/prof_${TAG}_$name -o run -- python3 $REPO/bench.py "$@" \
     > $REPO/gpurun_out/prof_${TAG}_$name/bench.log 2>&1) || { tail -30 gpurun_out/prof_${TAG}_$name/bench.log; return 1; }
  f=$(find gpurun_out/prof_${TAG}_$name -name "*kernel_stats.csv" | head -1)
  python scripts/prof_summary.py "$f" --steps $tot > gpurun_out/prof_${TAG}_$name/summary.txt && head -32 gpurun_out/prof_${TAG}_$name/summary.txt
}
if [[ $WHAT == all || $WHAT == gpt2 ]]; then
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_${TAG}_gpt2.log 2>&1 \
    || { tail -30 gpurun_out/bench_${TAG}_gpt2.log; exit 1; }
  tail -1 gpurun_out/bench_${TAG}_gpt2.log
  prof gpt2 5 --steps 3 --warmup 2 || exit 1
fi
if [[ $WHAT == all || $WHAT == llama ]]; then
  timeout -k 10 400 python bench.py --model llama2-7b --seq-len 4096 --micro-batch 4 --steps 4 --warmup 2 \
    > gpurun_out/bench_${TAG}_llama.log 2>&1 || { tail -30 gpurun_out/bench_${TAG}_llama.log; exit 1; }
  tail -1 gpurun_out/bench_${TAG}_llama.log
  prof llama 3 --model llama2-7b --seq-len 4096 --micro-batch 4 --steps 2 --warmup 1 || exit 1
fi
