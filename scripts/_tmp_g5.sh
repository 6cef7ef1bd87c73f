set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash scripts/gpu_tests.sh r03h tests || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r03h_bench.log 2>&1; tail -1 gpurun_out/r03h_bench.log | cut -c1-400
bash scripts/prof_ab.sh r03h "ORION_GEMM=auto" > gpurun_out/r03h_prof.log 2>&1; head -40 gpurun_out/r03h_prof.log
