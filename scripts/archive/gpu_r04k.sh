#!/bin/bash
# quad with loader waves: tests, bitwise A/B against the solver without them, timing, stamps
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r04k}
mkdir -p gpurun_out/$TAG
OUT=gpurun_out/$TAG/quad_loaders.txt
: > $OUT
PKG=$PWD/non-iid-distributed-learning-with-optimal-mixture-weights_amd
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "quad or prefetch or dropin_fedamw or config2" > gpurun_out/$TAG/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/$TAG/tests.log; exit 1; }
tail -1 gpurun_out/$TAG/tests.log
run() {   # env-assignments label N C NV EP
  env $1 timeout -k 10 120 python -u scripts/mix_time.py $3 $4 $5 $6 64 >> $OUT 2>&1 \
    || { echo "mix_time rc=$? ($2)"; tail -20 $OUT; exit 1; }
  echo "  ^ $2" >> $OUT
}
run "FS_MIX_QUAD_LOADERS=-1 FS_MIX_DUMP=gpurun_out/$TAG/prev.npy" "no loaders" 100 10 12800 10 || exit 1
run "FS_MIX_DUMP=gpurun_out/$TAG/new.npy" "loaders (default)" 100 10 12800 10 || exit 1
python -c "import numpy as np; a = np.load('gpurun_out/$TAG/prev.npy'); b = np.load('gpurun_out/$TAG/new.npy'); print('bitwise p/buf equal:', np.array_equal(a, b))" >> $OUT
run "FS_MIX_QUAD_LOADERS=-1" "no loaders" 100 10 12800 10 || exit 1
run "FS_MIX_PF_H=-1" "loaders, no helpers" 100 10 12800 10 || exit 1
run "FS_MIX_PF_H=8" "loaders, 8 helpers" 100 10 12800 10 || exit 1
run "FEDSIM_LIB=$PKG/libfedsim_stamps.so" "loaders, stamps" 100 10 12800 10 || exit 1
run "" "loaders (default) again" 100 10 12800 10 || exit 1
grep -v amdgpu.ids $OUT
