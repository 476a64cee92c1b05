#!/bin/bash
# Diagnostic builds (never shipped): libfedsim_<name>.so from a patched copy of csrc/ (a python
# patch file editing mixture.hip), linked with the tree's other objects.
#   scripts/build_mix_variant.sh <name> <patch.py>
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/non-iid-distributed-learning-with-optimal-mixture-weights_amd
NAME=$1; PATCH=$2
T=/tmp/mixvar_$NAME
rm -rf $T && mkdir -p $T/pkg/csrc $T/include && cp $PKG/csrc/*.hip $PKG/csrc/*.h $T/pkg/csrc/ && cp $ROOT/include/*.h $T/include/
python3 $PATCH $T/pkg/csrc/mixture.hip
(cd $T/pkg/csrc && /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -munsafe-fp-atomics \
  -c mixture.hip -o $T/mixture.o)
OBJS=$(cd $PKG/csrc/build && ls *.o | grep -v -E "^mixture|_stamps|_probe" | sed "s|^|$PKG/csrc/build/|")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $PKG/libfedsim_$NAME.so $OBJS $T/mixture.o -lpthread
echo built $PKG/libfedsim_$NAME.so
