# rocprofv3 kernel times of the phased GEMM's epilogue variants on the GPT-2 fc shape
# (65536 x 3072 x 768): store / bias / bias+GELU (forward), store / GELU-backward (dgrad);
# usage: bash scripts/experiments/epi_prof.sh [prefix]   (env, e.g. ORION_GEMM_PERSIST, passes through)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
P=${1:-}
run() { tag=$P$1; shift; timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/epi/$tag -o out -- python3 $R/scripts/gemm_one.py "$@" > $R/gpurun_out/epi_$tag.log 2>&1 || return 1; }
run s_dgrad 65536 3072 768 1 0 20 && run g_dgrad 65536 3072 768 1 3 20 && run s_fwd 65536 3072 768 0 0 20 && run g_fwd 65536 3072 768 0 2 20 && run b_fwd 65536 3072 768 0 1 20
