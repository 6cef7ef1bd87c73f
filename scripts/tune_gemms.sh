#!/bin/bash
# Tune hipBLASLt/rocBLAS solution choice for every GEMM shape of the GPT-2 bench with
# PyTorch TunableOp; the table is written to gpurun_out/tunableop/ and committed to
# orion_amd/tuning/ so bench runs load it (no tuning at bench time).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/tunableop
export HSA_ENABLE_IPC_MODE_LEGACY=0
export PYTORCH_TUNABLEOP_ENABLED=1
export PYTORCH_TUNABLEOP_TUNING=1
export PYTORCH_TUNABLEOP_VERBOSE=1
export PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop/tunableop_results.csv
export PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=${TUNE_MS:-60}
ARGS=${@:-"--steps 2 --warmup 1"}
timeout -k 10 1000 python bench.py $ARGS --no-tuned-gemms > gpurun_out/tunableop/tune.log 2>&1
rc=$?
tail -3 gpurun_out/tunableop/tune.log
ls -la gpurun_out/tunableop/
exit $rc
