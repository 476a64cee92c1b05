#!/bin/bash
# Diagnostic build (never shipped): the library with the pipe form's wave-priority experiment
# -DPP_PRIO=M (0: none; 1: the SIMDs second waves at priority 1; 2 (shipped): the hand-off phases at priority 3;
# 3: both).   scripts/build_pipe_prio_variant.sh M  ->  <pkg>/libfedsim_pipeprio<M>.so
set -e
M=$1
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/non-iid-distributed-learning-with-optimal-mixture-weights_amd
H="/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -munsafe-fp-atomics"
mkdir -p /tmp/pipe_prio_$M
(cd $PKG/csrc && $H -DPP_PRIO=$M -c local_train_pipe.hip -o /tmp/pipe_prio_$M/ltp.o)
objs=""
for f in local_train local_train_split local_train_pair aggregate eval mixture mix_z randperm round feature_map gram; do
  objs="$objs $PKG/csrc/build/$f.o"
done
$H -shared -o $PKG/libfedsim_pipeprio$M.so /tmp/pipe_prio_$M/ltp.o $objs $PKG/csrc/build/host.o $PKG/csrc/build/libsvm.o -lpthread
echo built $PKG/libfedsim_pipeprio$M.so
