#!/bin/bash
# quad loader-wave variants: register-ring classes 3 (shipped) vs 2 / 1 (libfedsim_ql{2,1}.so,
# built from patched copies), config 2 p-solve shape; bitwise dumps compared
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-qlv}
mkdir -p gpurun_out/$TAG
OUT=gpurun_out/$TAG/qlv.txt
: > $OUT
PKG=$PWD/non-iid-distributed-learning-with-optimal-mixture-weights_amd
for rep in 1 2; do
  for lib in libfedsim.so libfedsim_ql2.so libfedsim_ql1.so; do
    FEDSIM_LIB=$PKG/$lib FS_MIX_DUMP=gpurun_out/$TAG/$lib.npy timeout -k 10 120 python -u scripts/mix_time.py 100 10 12800 10 64 >> $OUT 2>&1 \
      || { echo "mix_time rc=$? ($lib)"; tail -20 $OUT; exit 1; }
    echo "  ^ $lib" >> $OUT
  done
done
python -c "
import numpy as np
a = np.load('gpurun_out/$TAG/libfedsim.so.npy')
for v in ('ql2', 'ql1'):
    print(v, 'bitwise equal:', np.array_equal(a, np.load('gpurun_out/$TAG/libfedsim_%s.so.npy' % v)))" >> $OUT
grep -v amdgpu.ids $OUT
