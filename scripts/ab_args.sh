#!/bin/bash
# Same-box alternating A/B of two bench.py argument sets.
# usage: scripts/ab_args.sh NAME "ARGS_A" "ARGS_B" REPS   (common args: --steps 30 --warmup 5)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
name=$1; A=$2; B=$3; reps=$4
mkdir -p gpurun_out
out=gpurun_out/ab_$name.log; : > "$out"
for i in $(seq 1 "$reps"); do
  for v in A B; do
    a=$A; [[ $v == B ]] && a=$B
    # shellcheck disable=SC2086
    r=$(timeout -k 10 300 python bench.py --steps 30 --warmup 5 $a 2>"gpurun_out/ab_${name}_err.log" | tail -1) \
      || { echo "run failed ($v)"; tail -20 "gpurun_out/ab_${name}_err.log"; exit 1; }
    ms=$(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')
    echo "$v [$a] $ms" | tee -a "$out"
  done
done
