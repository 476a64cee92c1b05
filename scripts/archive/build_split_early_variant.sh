#!/bin/bash
# Diagnostic build (never shipped): the library with the split form's early-issue depth set to N
# row loads -- for the PROX instances (KIND = prox, default) or the others (KIND = plain) -- an A/B
# of the depth.  Built from a patched copy of csrc/ in /tmp (the tree's sources stay untouched).
#   scripts/build_split_early_variant.sh N [prox|plain]  ->  <pkg>/libfedsim_<kind>early<N>.so
set -e
N=$1
KIND=${2:-prox}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/non-iid-distributed-learning-with-optimal-mixture-weights_amd
B=/tmp/split_early_${KIND}_$N
T=$B/pkg/csrc
rm -rf $B && mkdir -p $T $B/include
cp $PKG/csrc/*.hip $PKG/csrc/*.h $T/ && cp $ROOT/include/*.h $B/include/
python3 - $T/local_train_split.hip $N $KIND <<'PY'
import sys
p, n, kind = sys.argv[1], sys.argv[2], sys.argv[3]; s = open(p).read()
if kind == 'prox':
    a = "  if (P.prox && early) launch_split_s<RT, G, true, EARLY_PROX, 1>(P, X, grid, lds, st);"
    b = "  if (P.prox && early) launch_split_s<RT, G, true, %s, 1>(P, X, grid, lds, st);" % n
else:
    a = "  else if (early) launch_split_s<RT, G, false, EARLY_G, 1>(P, X, grid, lds, st);"
    b = "  else if (early) launch_split_s<RT, G, false, %s, 1>(P, X, grid, lds, st);" % n
assert s.count(a) == 1, 'patch point moved'
open(p, 'w').write(s.replace(a, b))
PY
cd $T
H="/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -munsafe-fp-atomics"
mkdir -p build
$H -c local_train_split.hip -o build/lts.o
objs=""
for f in local_train local_train_pair local_train_pipe aggregate eval mixture mix_z randperm round feature_map gram; do
  objs="$objs $PKG/csrc/build/$f.o"
done
$H -shared -o $PKG/libfedsim_${KIND}early$N.so build/lts.o $objs $PKG/csrc/build/host.o $PKG/csrc/build/libsvm.o -lpthread
echo built $PKG/libfedsim_${KIND}early$N.so
