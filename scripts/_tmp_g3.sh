set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash scripts/gpu_tests.sh r03e tests/test_gemm_gpu.py && \
timeout -k 10 300 python scripts/bench_gemm.py --iters 20 --cfgs 9 --check > gpurun_out/r03e_gemm.log 2>&1; tail -13 gpurun_out/r03e_gemm.log
for i in 1 2 3; do
 for v in "ORION_GEMM=blas" "ORION_GEMM=auto" "ORION_GEMM=auto ORION_FUSED_MLP=1" "ORION_GEMM=hip ORION_FUSED_MLP=1"; do
  r=$(env $v timeout -k 10 300 python bench.py --steps 20 --warmup 5 2>/dev/null | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])') || { echo "fail $v"; exit 1; }
  echo "[$v] $r" | tee -a gpurun_out/r03e_ab.log
 done
done
