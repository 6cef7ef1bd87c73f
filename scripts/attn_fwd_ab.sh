set -o pipefail
cd /root/repo
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/attn_tests.log 2>&1 || { tail -30 gpurun_out/attn_tests.log; exit 1; }
tail -2 gpurun_out/attn_tests.log
for r in 1 2 3; do
  for v in v2 v3; do
    ORION_ATTN_FWD=$v timeout -k 10 120 python scripts/attn_fwd_time.py 64 1024 12 12 64 || exit 1
    ORION_ATTN_FWD=$v timeout -k 10 120 python scripts/attn_fwd_time.py 4 4096 32 32 128 || exit 1
  done
done
