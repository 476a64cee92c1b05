#!/bin/bash
# Diagnostic builds (never shipped): libfedsim_<name>.so with ONE device source replaced by a
# patched copy (a python patch file editing csrc/<file>), linked with the tree's other objects.
#   scripts/build_variant.sh <name> <file.hip> <patch.py> [more patch.py ...]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/non-iid-distributed-learning-with-optimal-mixture-weights_amd
NAME=$1; FILE=$2; shift 2
T=/tmp/variant_$NAME
rm -rf $T && mkdir -p $T/pkg/csrc $T/include && cp $PKG/csrc/*.hip $PKG/csrc/*.h $T/pkg/csrc/ && cp $ROOT/include/*.h $T/include/
for P in "$@"; do python3 $P $T/pkg/csrc/$FILE; done
BASE=${FILE%.hip}
(cd $T/pkg/csrc && /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result \
  -munsafe-fp-atomics -c $FILE -o $T/$BASE.o)
OBJS=$(cd $PKG/csrc/build && ls *.o | grep -v -E "^$BASE\.o$|_stamps|_probe" | sed "s|^|$PKG/csrc/build/|")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $PKG/libfedsim_$NAME.so $OBJS $T/$BASE.o -lpthread
echo built $PKG/libfedsim_$NAME.so
