#!/bin/bash
# usage: ab_env.sh NAME "ENV_A" "ENV_B" reps bench-args...
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
name=$1; A=$2; B=$3; reps=$4; shift 4
mkdir -p gpurun_out
out=gpurun_out/ab_$name.log; : > $out
for i in $(seq 1 $reps); do
  for v in A B; do
    e=$A; [[ $v == B ]] && e=$B
    r=$(env $e timeout -k 10 300 python bench.py "$@" 2>gpurun_out/ab_${name}_err.log | tail -1) || { echo "run failed ($v)"; tail -20 gpurun_out/ab_${name}_err.log; exit 1; }
    ms=$(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')
    echo "$v [$e] $ms" | tee -a $out
  done
done
