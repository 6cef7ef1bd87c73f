export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_b5.log 2>&1 && \
bash scripts/attn_ab.sh pf2 ORION_ATTN_KV_PF2=1 ORION_ATTN_KV_PF2=0 ORION_ATTN_KV_PF2=1 ORION_ATTN_KV_PF2=0 > /dev/null && \
bash scripts/ab_env.sh kv_pf2 "ORION_ATTN_KV_PF2=1" "ORION_ATTN_KV_PF2=0" 3 --steps 20 --warmup 5
