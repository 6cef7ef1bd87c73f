export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 120 python scripts/attn_stamps.py > gpurun_out/stamps_new.log 2>&1 && \
ORION_AMD_EXT=$PWD/variants/_C_head.so timeout -k 10 120 python scripts/attn_stamps.py > gpurun_out/stamps_head.log 2>&1
