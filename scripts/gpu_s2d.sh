#!/bin/bash
# register p-solve with the fold-once update: GPU suite, then timing (plain + stamps) at
# config 2 and other register-solver shapes.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r02s2d}; mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step pytest timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
tail -2 $O/gpu_tests.log
for a in "100 10 12800 10" "100 10 512 250" "64 7 12800 10" "200 4 12800 10" "128 10 12800 10"; do
  FS_MIX_SOLVER=reg step "plain $a" timeout -k 10 120 python -u scripts/mix_time.py $a >> $O/time.log 2>&1
  FS_MIX_SOLVER=reg FEDSIM_LIB=$PWD/non-iid-distributed-learning-with-optimal-mixture-weights_amd/libfedsim_stamps.so step "stamps $a" timeout -k 10 120 python -u scripts/mix_time.py $a >> $O/time.log 2>&1
done
for h in 2 4; do FS_MIX_SOLVER=reg FS_MIX_PF_H=$h step "pf $h" timeout -k 10 120 python -u scripts/mix_time.py 100 10 12800 10 >> $O/time.log 2>&1; done
grep -E 'mix_solve|ticks' $O/time.log
