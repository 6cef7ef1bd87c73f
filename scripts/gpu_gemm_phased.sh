#!/bin/bash
# Phased GEMM: numerics tests, then microbench vs the 2-stage kernel and hipBLASLt.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py > gpurun_out/gemm_phased_tests.log 2>&1 || { tail -30 gpurun_out/gemm_phased_tests.log; exit 1; }
tail -3 gpurun_out/gemm_phased_tests.log
timeout -k 10 400 python -u scripts/bench_gemm.py --cfgs 7,0 --square 4096 --check --iters 15 > gpurun_out/gemm_phased_bench.log 2>&1
rc=$?; cat gpurun_out/gemm_phased_bench.log; exit $rc
