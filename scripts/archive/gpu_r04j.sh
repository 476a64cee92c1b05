#!/bin/bash
# p-solve instruction trims (fused row max, interleaved logit chains, branch-free momentum, one
# hazard pad per reduce-scatter level): bitwise A/B against the previous build
# (libfedsim_prev.so), timing, stamps, mix parity tests.   scripts/gpu_r04j.sh <tag>
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r04j}
mkdir -p gpurun_out/$TAG
OUT=gpurun_out/$TAG/psolve_trim.txt
: > $OUT
PKG=$PWD/non-iid-distributed-learning-with-optimal-mixture-weights_amd
run() {   # lib dumpname N C NV EP
  env ${1:+FEDSIM_LIB=$1} FS_MIX_DUMP=gpurun_out/$TAG/$2.npy timeout -k 10 120 python -u scripts/mix_time.py $3 $4 $5 $6 64 \
    >> $OUT 2>&1 || { echo "mix_time rc=$? ($2)"; tail -20 $OUT; exit 1; }
  echo "  ^ $2" >> $OUT
}
for sh in "c2 100 10 12800 10" "c5 1000 10 32000 5" "n300 300 10 12800 5"; do
  set -- $sh
  run $PKG/libfedsim_prev.so prev_$1 $2 $3 $4 $5 || exit 1
  run "" new_$1 $2 $3 $4 $5 || exit 1
  python -c "import numpy as np, sys; a = np.load('gpurun_out/$TAG/prev_$1.npy'); b = np.load('gpurun_out/$TAG/new_$1.npy'); print('$1 bitwise p/buf equal:', np.array_equal(a, b), 'max |diff|', float(np.abs(a - b).max()))" >> $OUT
done
run $PKG/libfedsim_stamps.so st_c2 100 10 12800 10 || exit 1
run $PKG/libfedsim_stamps.so st_c5 1000 10 32000 5 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread \
  -k "mix or horizon or fedamw" > gpurun_out/$TAG/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/$TAG/tests.log; exit 1; }
tail -1 gpurun_out/$TAG/tests.log
grep -v amdgpu.ids $OUT
