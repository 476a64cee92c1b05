#!/bin/bash
# quad p-solver: issue split sweep (parity at split 3/5, timing 10/7/5/3, with/without helpers)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r02s2j}; mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
for sp in 3 5; do
FS_MIX_QUAD_SPLIT=$sp step "tests split $sp" timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "quad" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests_$sp.log 2>&1
tail -1 $O/tests_$sp.log
done
SL=$PWD/non-iid-distributed-learning-with-optimal-mixture-weights_amd/libfedsim_stamps.so
for cfg in "10 0" "7 0" "5 0" "3 0" "10 4" "5 4" "3 4"; do set -- $cfg
  FS_MIX_SOLVER=quad FS_MIX_QUAD_SPLIT=$1 FS_MIX_PF_H=$2 step "split $1 pf $2" timeout -k 10 120 python -u scripts/mix_time.py 100 10 12800 10 >> $O/time.log 2>&1
  tail -2 $O/time.log | head -1
done
for sp in 5 3; do
FS_MIX_SOLVER=quad FS_MIX_QUAD_SPLIT=$sp FEDSIM_LIB=$SL step "stamps $sp" timeout -k 10 120 python -u scripts/mix_time.py 100 10 12800 10 >> $O/time.log 2>&1
grep ticks $O/time.log | tail -1
done
