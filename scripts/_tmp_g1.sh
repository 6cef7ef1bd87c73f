set -o pipefail
bash scripts/gpu_tests.sh r03c tests/test_gemm_gpu.py && \
timeout -k 10 300 python scripts/bench_gemm.py --iters 20 --square 4096 --cfgs 9,7 --check > gpurun_out/r03c_gemm.log 2>&1; tail -20 gpurun_out/r03c_gemm.log
