#!/bin/bash
# Build variants/_C_<name>.so: the in-tree objects with ONE source recompiled under extra
# flags (A/B and bisection builds; scripts/ab_variants.sh runs them).
# usage: scripts/build_variant.sh NAME SOURCE.hip "-DFLAG ..."
set -e
cd "$(dirname "$0")/.."
NAME=$1; SRC=$2; FLAGS=$3
HIPCC=/opt/rocm/bin/hipcc
TL=$(python -c "import torch,os;print(os.path.join(os.path.dirname(torch.__file__),'lib'))")
mkdir -p variants build/variants
base=$(basename $SRC)
$HIPCC -x hip --offload-arch=gfx950 -munsafe-fp-atomics -O3 -std=c++17 -fPIC -Icsrc $FLAGS \
  -c $SRC -o build/variants/${base}_$NAME.o
objs=$(ls build/csrc/*.o | grep -v "/$base.o")
$HIPCC -shared -fPIC --offload-arch=gfx950 $objs build/variants/${base}_$NAME.o -o variants/_C_$NAME.so \
  -L$TL -lc10 -lc10_hip -ltorch -ltorch_cpu -ltorch_hip -Wl,-rpath,$TL
echo variants/_C_$NAME.so
