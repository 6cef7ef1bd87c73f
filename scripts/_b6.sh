export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_b6.log 2>&1 && \
bash scripts/attn_ab.sh wait "ORION_ATTN_KV_NW=4" "ORION_ATTN_KV_NW=8" "ORION_ATTN_KV_NW=4 ORION_ATTN_KV_PF2=1" "ORION_ATTN_KV_NW=4" "ORION_ATTN_KV_NW=8" > /dev/null && \
ROUNDS=3 AB_TIMEOUT=200 bash scripts/ab_variants.sh python bench.py --steps 20 --warmup 5 > gpurun_out/abv_b6.log 2>&1
