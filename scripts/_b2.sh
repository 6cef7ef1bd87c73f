export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
bash scripts/ab_env.sh shortk_fwd "ORION_GEMM_SHORTK_FWD=1" "ORION_GEMM_SHORTK_FWD=0" 3 --steps 20 --warmup 5 && \
bash scripts/profile.sh --steps 6 --warmup 3 > gpurun_out/prof_b2.log 2>&1 && \
python scripts/prof_summary.py gpurun_out/prof/run_kernel_trace.csv --steady > gpurun_out/prof_b2_steady.txt 2>&1
