set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python scripts/bench_gemm.py --llama --M 16384 --iters 10 --cfgs 9 > gpurun_out/r03i_gemm_llama.log 2>&1; tail -11 gpurun_out/r03i_gemm_llama.log
for v in "ORION_GEMM=blas" "ORION_GEMM=auto"; do
  env $v timeout -k 10 400 python bench.py --model llama2-7b --seq-len 4096 --steps 4 --warmup 2 > gpurun_out/r03i_llama_$v.log 2>&1 || { tail -5 gpurun_out/r03i_llama_$v.log; exit 1; }
  echo "[$v] $(tail -1 gpurun_out/r03i_llama_$v.log | cut -c1-330)"
done
timeout -k 10 400 python bench.py --model llama2-7b --seq-len 4096 --steps 4 --warmup 2 --zero1 > gpurun_out/r03i_llama_zero1.log 2>&1 || { tail -5 gpurun_out/r03i_llama_zero1.log; exit 1; }
tail -1 gpurun_out/r03i_llama_zero1.log
