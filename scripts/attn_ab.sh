#!/bin/bash
# Attention kernel A/B on the GPT-2 and Llama-7B shapes: bench_attn.py under each env setting.
# usage: scripts/attn_ab.sh TAG "ENV1" "ENV2" ...   (e.g. "ORION_ATTN_BWD64=0")
set -o pipefail
cd "$(dirname "$0")/.."
TAG=$1; shift
OUT=gpurun_out/attn_ab_$TAG.log
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
: > $OUT
for e in "$@"; do
  for shape in "--B 64 --T 1024 --H 12 --D 64" "--B 4 --T 4096 --H 32 --D 128"; do
    echo "[$e] $shape $(env $e timeout -k 10 120 python3 scripts/bench_attn.py $shape --iters 30)" >> $OUT || exit 1
  done
done
cat $OUT
