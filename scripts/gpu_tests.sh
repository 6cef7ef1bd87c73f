#!/bin/bash
# GPU tests (optionally a -k filter / file list) under a time limit, log in gpurun_out/.
# usage: scripts/gpu_tests.sh TAG [pytest args...]
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-t}; shift
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -m gpu -x -v --timeout 240 --timeout-method thread "$@" \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_$TAG.log
exit $rc
