#!/bin/bash
# Diagnostic build (never shipped): the library with the split form's early-issue depth for the
# PROX instances set to N row loads (the shipped depth is the width's EARLY_G) -- an A/B of the
# depth at config 3.  Built from a patched copy of csrc/ in /tmp (the tree's sources stay untouched).
#   scripts/build_split_early_variant.sh N   ->  <pkg>/libfedsim_proxearly<N>.so
set -e
N=$1
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/non-iid-distributed-learning-with-optimal-mixture-weights_amd
T=/tmp/split_early_$N/pkg/csrc
rm -rf /tmp/split_early_$N && mkdir -p $T /tmp/split_early_$N/include
cp $PKG/csrc/*.hip $PKG/csrc/*.h $T/ && cp $ROOT/include/*.h /tmp/split_early_$N/include/
python3 - $T/local_train_split.hip $N <<'PY'
import sys
p, n = sys.argv[1], sys.argv[2]; s = open(p).read()
a = "  if (P.prox && early) launch_split_s<RT, G, true, EARLY_G, 1>(P, X, grid, lds, st);"
assert s.count(a) == 1, 'patch point moved'
s = s.replace(a, "  if (P.prox && early) launch_split_s<RT, G, true, %s, 1>(P, X, grid, lds, st);" % n)
open(p, 'w').write(s)
PY
cd $T
H="/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -munsafe-fp-atomics"
mkdir -p build
$H -c local_train_split.hip -o build/lts.o
objs=""
for f in local_train local_train_pair local_train_pipe aggregate eval mixture mix_z randperm round feature_map gram; do
  objs="$objs $PKG/csrc/build/$f.o"
done
$H -shared -o $PKG/libfedsim_proxearly$N.so build/lts.o $objs $PKG/csrc/build/host.o $PKG/csrc/build/libsvm.o -lpthread
echo built $PKG/libfedsim_proxearly$N.so
