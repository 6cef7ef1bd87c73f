set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
ORION_GEMM16_KS=1 bash scripts/gpu_tests.sh r03g tests/test_gemm_gpu.py || exit 1
timeout -k 10 300 python scripts/bench_gemm.py --iters 20 --square 4096 --cfgs 9ks,9 --check > gpurun_out/r03g_gemm.log 2>&1; tail -14 gpurun_out/r03g_gemm.log
for sh in "4096 4096 4096 0 1" "65536 2304 768 0 1" "65536 768 3072 1 1"; do
  timeout -k 10 120 python scripts/gemm16_stamps.py $sh >> gpurun_out/r03g_stamps.log 2>&1 || break
done; cat gpurun_out/r03g_stamps.log
