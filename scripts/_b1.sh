export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_kernels_gpu.py tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_b1.log 2>&1 && \
timeout -k 10 300 python scripts/bench_gemm.py --cfgs p,t,s --check > gpurun_out/bg_pts.log 2>&1 && \
timeout -k 10 200 python scripts/coresidency.py > gpurun_out/cores.log 2>&1 && \
bash scripts/attn_ab.sh pair ORION_ATTN_PAIR=1 ORION_ATTN_PAIR=0 ORION_ATTN_PAIR=1 ORION_ATTN_PAIR=0
