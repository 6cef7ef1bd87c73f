set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out/r03a
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r03a/bench.log 2>&1 && tail -1 gpurun_out/r03a/bench.log &&
timeout -k 10 400 python scripts/bench_gemm.py --iters 20 --square 4096 > gpurun_out/r03a/gemm.log 2>&1 && cat gpurun_out/r03a/gemm.log | tail -20
