export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_b3.log 2>&1 && \
bash scripts/attn_ab.sh fast ORION_ATTN_FWD_FAST=1 ORION_ATTN_FWD_FAST=0 ORION_ATTN_FWD_FAST=1 ORION_ATTN_FWD_FAST=0
