export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_b4.log 2>&1 && \
bash scripts/attn_ab.sh fastcb "ORION_ATTN_FWD_FAST=1 ORION_ATTN_DQ_CB=1" "ORION_ATTN_FWD_FAST=0 ORION_ATTN_DQ_CB=0" "ORION_ATTN_FWD_FAST=1 ORION_ATTN_DQ_CB=0" "ORION_ATTN_FWD_FAST=1 ORION_ATTN_DQ_CB=1" "ORION_ATTN_FWD_FAST=0 ORION_ATTN_DQ_CB=0" > /dev/null && \
ROUNDS=3 AB_TIMEOUT=200 bash scripts/ab_variants.sh python bench.py --steps 20 --warmup 5 > gpurun_out/abv_b4.log 2>&1
