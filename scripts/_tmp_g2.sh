set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python scripts/bench_wgrad_cfg.py --cfgs 9,7 > gpurun_out/r03d_wgrad.log 2>&1; tail -8 gpurun_out/r03d_wgrad.log
timeout -k 10 300 python scripts/bench_wgrad_cfg.py --cfgs 9,7 --M 16384 --shapes 12288x4096,4096x4096,22016x4096,4096x11008,32000x4096 > gpurun_out/r03d_wgrad_llama.log 2>&1; tail -8 gpurun_out/r03d_wgrad_llama.log
bash scripts/ab_env.sh wg16 "ORION_WGRAD_CFG=7" "ORION_WGRAD_CFG=9" 3 --steps 20 --warmup 5
for sh in "4096 4096 4096 0" "65536 2304 768 0" "65536 768 3072 0" "65536 768 3072 1" "65536 50304 768 0"; do
  timeout -k 10 120 python scripts/gemm16_stamps.py $sh >> gpurun_out/r03d_stamps.log 2>&1 || break
done; cat gpurun_out/r03d_stamps.log
