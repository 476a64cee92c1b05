#!/bin/bash
# round 6 (session 2): the pipe form's swizzled partial-logit slots -- its bitwise tests, then
# config 4's launch (the planner's pipe form) against the previous build (base.so), interleaved
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
PKG=non-iid-distributed-learning-with-optimal-mixture-weights_amd
O=gpurun_out/r06pz; mkdir -p $O; rm -f $O/ab.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipe.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || exit $rc
for k in 1 2 3 4; do
  for lib in libfedsim base; do
    FEDSIM_LIB=$PKG/$lib.so timeout -k 10 120 python -u scripts/lt_sweep.py --config 4 --G 0 --reg 0 --reps 30 >> $O/ab.txt 2>&1 || exit 1
    echo "^ c4 $lib" >> $O/ab.txt
  done
done
grep -v amdgpu.ids $O/ab.txt
