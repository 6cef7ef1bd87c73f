#!/bin/bash
# Continuous-integration pipeline (the role of the reference's tox.ini / .travis.yml envs),
# CPU stages on any host with the ROCm toolchain; the GPU stage needs an MI355X.
#   build   : hipcc cross-compile of every csrc/*.hip for gfx950 (forced) + package import
#   lint    : scripts/lint.py (compile, unused imports, whitespace, line length, bare except)
#   test    : pytest -m "not gpu" (unit, multi-process gloo DDP, functional CLI, ASan/UBSan host)
#   demo    : the reference's demo_random env: random search on the demo black box
#   gpu     : pytest -m gpu + smoke (run on the GPU box, e.g. through gpurun)
# usage: scripts/ci.sh [build lint test demo gpu]   (default: build lint test demo)
set -euo pipefail
cd "$(dirname "$0")/.."
STAGES=${*:-build lint test demo}
for stage in $STAGES; do
  echo "=== $stage"
  case $stage in
    build) python -c "import __graft_entry__ as g; g.build()" ;;
    lint) python scripts/lint.py ;;
    test) python -m pytest tests -x -q -m "not gpu" -n 4 --timeout 900 ;;
    demo)
      tmp=$(mktemp -d)
      (cd tests/functional/demo && METAOPT_DB_TYPE=sqlite METAOPT_DB_ADDRESS=$tmp/demo.sqlite \
         XDG_CONFIG_HOME=$tmp python ../../../bin/orion -n ci_demo_random --max-trials 20 \
         --pool-size 5 ./black_box.py "-x~normal(30, 5)")
      rm -rf "$tmp" ;;
    gpu)
      export HSA_ENABLE_IPC_MODE_LEGACY=0
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    *) echo "unknown stage $stage"; exit 2 ;;
  esac
done
echo "ci: all stages passed ($STAGES)"
