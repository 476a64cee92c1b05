#!/bin/bash
# Diagnostic A/B build (never shipped): libfedsim with ONE source recompiled under extra -D flags.
#   scripts/build_variant.sh <source.hip> <out-name> -DFOO=1 [...]  ->  <pkg>/<out-name>.so
# Load it with FEDSIM_LIB=<pkg>/<out-name>.so (scripts/lt_sweep.py, bench.py).
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/non-iid-distributed-learning-with-optimal-mixture-weights_amd
SRC=$1; OUT=$2; shift 2
make -s -C $PKG/csrc
H="/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -munsafe-fp-atomics"
base=$(basename $SRC .hip)
$H "$@" -c $PKG/csrc/$SRC -o $PKG/csrc/build/variant_${OUT}_$base.o
objs=$(ls $PKG/csrc/build/*.o | grep -v -e "/$base.o" -e variant_ -e _stamps -e _probe)
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $PKG/$OUT.so $objs $PKG/csrc/build/variant_${OUT}_$base.o -lpthread
echo built $PKG/$OUT.so
