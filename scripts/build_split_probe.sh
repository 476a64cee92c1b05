#!/bin/bash
# Diagnostic build (never shipped): the split-client local-training kernel WITHOUT its in-loop
# row loads (each wave keeps training on the rows of its first step: wrong weights, timing
# only), with the phase stamps -- what a step costs without the row stream.  Built from a
# patched copy of csrc/ in /tmp so the tree's sources (and their PMC revision) stay untouched.
#   scripts/build_split_probe.sh   ->  <pkg>/libfedsim_split_probe_stamps.so
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/non-iid-distributed-learning-with-optimal-mixture-weights_amd
T=/tmp/split_probe/pkg/csrc                      # (common.h includes ../../include/fedsim.h)
rm -rf /tmp/split_probe && mkdir -p $T /tmp/split_probe/include
cp $PKG/csrc/*.hip $PKG/csrc/*.h $T/ && cp $ROOT/include/*.h /tmp/split_probe/include/
python3 - $T/local_train_split.hip <<'PY'
import sys
p = sys.argv[1]; s = open(p).read()
a = """        xf[i][kk >> 2][kk & 3] =
            ld4(P.phi + (int64_t)pn[kk >> 2] * ld + 64 * t0 + 4 * lg + 64 * (w + NW * i) + 16 * (kk & 3));"""
b = """                xf[i][kk >> 2][kk & 3] = ld4(P.phi + (int64_t)pn[kk >> 2] * ld + 64 * t0 + 4 * lg + 64 * Tl + 16 * (kk & 3));"""
assert s.count(a) == 1 and s.count(b) == 1, 'probe patch points moved'
s = s.replace(a, "        (void)i; (void)kk;").replace(b, "                (void)Tl;")
open(p, 'w').write(s)
PY
cd $T
H="/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -munsafe-fp-atomics"
mkdir -p build
$H -DFS_STAMPS -c local_train_split.hip -o build/lts.o
objs=""
for f in local_train local_train_pair aggregate eval mixture mix_z randperm round feature_map gram; do
  objs="$objs $PKG/csrc/build/$f.o"
done
$H -shared -o $PKG/libfedsim_split_probe_stamps.so build/lts.o $objs $PKG/csrc/build/host.o $PKG/csrc/build/libsvm.o -lpthread
echo built $PKG/libfedsim_split_probe_stamps.so
