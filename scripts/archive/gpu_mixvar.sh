#!/bin/bash
# p-solve variant A/B (libfedsim.so vs libfedsim_<v>.so from scripts/build_mix_variant.sh), one box,
# alternating, p/buf bitwise compared.   scripts/gpu_mixvar.sh <tag> "<N C NV EP>" <v1> [v2 ...]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=$1; SHAPE=$2; shift 2
mkdir -p gpurun_out/$TAG
OUT=gpurun_out/$TAG/ab.txt
: > $OUT
PKG=$PWD/non-iid-distributed-learning-with-optimal-mixture-weights_amd
for rep in 1 2; do
  for v in shipped "$@"; do
    lib=libfedsim.so; [ "$v" = shipped ] || lib=libfedsim_$v.so
    FEDSIM_LIB=$PKG/$lib FS_MIX_DUMP=gpurun_out/$TAG/$v.npy timeout -k 10 120 python -u scripts/mix_time.py $SHAPE 64 >> $OUT 2>&1 \
      || { echo "mix_time rc=$? ($v)"; tail -20 $OUT; exit 1; }
    echo "  ^ $v" >> $OUT
  done
done
for v in "$@"; do
  python -c "import numpy as np; print('$v bitwise equal:', np.array_equal(np.load('gpurun_out/$TAG/shipped.npy'), np.load('gpurun_out/$TAG/$v.npy')))" >> $OUT
done
grep -v amdgpu.ids $OUT
