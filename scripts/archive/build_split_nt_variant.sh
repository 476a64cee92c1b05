#!/bin/bash
set -e
ROOT=/root/repo
PKG=$ROOT/non-iid-distributed-learning-with-optimal-mixture-weights_amd
B=/tmp/split_nt
T=$B/pkg/csrc
rm -rf $B && mkdir -p $T $B/include
cp $PKG/csrc/*.hip $PKG/csrc/*.h $T/ && cp $ROOT/include/*.h $B/include/
python3 - $T <<'PY'
import sys
t = sys.argv[1]
c = open(t + '/common.h').read()
c = c.replace("__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }",
 "__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }\ntypedef float fs_v4f __attribute__((ext_vector_type(4)));\n__device__ __forceinline__ float4 ld4nt(const float* p) { const fs_v4f v = __builtin_nontemporal_load(reinterpret_cast<const fs_v4f*>(p)); return make_float4(v.x, v.y, v.z, v.w); }")
open(t + '/common.h', 'w').write(c)
s = open(t + '/local_train_split.hip').read()
a = "        xf[i][kk >> 2][kk & 3] =\n            ld4(P.phi"
assert a in s
s = s.replace(a, "        xf[i][kk >> 2][kk & 3] =\n            ld4nt(P.phi")
a = "                xf[i][kk >> 2][kk & 3] = ld4(P.phi"
assert a in s
s = s.replace(a, "                xf[i][kk >> 2][kk & 3] = ld4nt(P.phi")
open(t + '/local_train_split.hip', 'w').write(s)
PY
cd $T
H="/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -munsafe-fp-atomics"
mkdir -p build
$H -c local_train_split.hip -o build/lts.o
objs=""
for f in local_train local_train_pair local_train_pipe aggregate eval mixture mix_z randperm round feature_map gram; do objs="$objs $PKG/csrc/build/$f.o"; done
$H -shared -o $PKG/libfedsim_nt.so build/lts.o $objs $PKG/csrc/build/host.o $PKG/csrc/build/libsvm.o -lpthread
echo built
