#!/bin/bash
# qmc with loader waves: tests (bitwise vs without, blocked layout, horizons), timing on/off at
# config 5's shape and N = 300, stamps
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r04l}
mkdir -p gpurun_out/$TAG
OUT=gpurun_out/$TAG/qmc_loaders.txt
: > $OUT
PKG=$PWD/non-iid-distributed-learning-with-optimal-mixture-weights_amd
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "qmc or blocked or horizon or quad or config5" > gpurun_out/$TAG/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/$TAG/tests.log; exit 1; }
tail -1 gpurun_out/$TAG/tests.log
run() {   # env-assignments label N C NV EP
  env $1 timeout -k 10 120 python -u scripts/mix_time.py $3 $4 $5 $6 64 >> $OUT 2>&1 \
    || { echo "mix_time rc=$? ($2)"; tail -20 $OUT; exit 1; }
  echo "  ^ $2" >> $OUT
}
run "FS_MIX_QUAD_LOADERS=-1" "no loaders" 1000 10 32000 5 || exit 1
run "" "loaders (default)" 1000 10 32000 5 || exit 1
run "FS_MIX_PF_H=8" "loaders, 8 helpers" 1000 10 32000 5 || exit 1
run "FS_MIX_PF_H=-1" "loaders, no helpers" 1000 10 32000 5 || exit 1
run "FS_MIX_QUAD_LOADERS=-1" "no loaders" 300 10 12800 5 || exit 1
run "" "loaders (default)" 300 10 12800 5 || exit 1
run "FEDSIM_LIB=$PKG/libfedsim_stamps.so" "loaders, stamps" 1000 10 32000 5 || exit 1
run "" "loaders (default) again" 1000 10 32000 5 || exit 1
grep -v amdgpu.ids $OUT
