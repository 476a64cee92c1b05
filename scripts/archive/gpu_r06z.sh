#!/bin/bash
# round 6 (session 2): the narrow chained instances' row-prefetch helpers (ABI 17,
# fs_tuning.split_prefetch): bitwise tests, then config 1's launch with and without them
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06z; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_split_early.py tests/test_abi.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || exit $rc
PKG=non-iid-distributed-learning-with-optimal-mixture-weights_amd
for k in 1 2; do
  for pf in off on; do
    timeout -k 10 120 python -u scripts/lt_sweep.py --config 1 --G 8 --prefetch $pf >> $O/ab.txt 2>&1 || exit 1
    echo "^ c1 prefetch $pf (lead 2)" >> $O/ab.txt
  done
  FEDSIM_LIB=$PKG/pflead4.so timeout -k 10 120 python -u scripts/lt_sweep.py --config 1 --G 8 --prefetch on >> $O/ab.txt 2>&1 || exit 1
  echo "^ c1 prefetch on, lead 4" >> $O/ab.txt
done
grep -v amdgpu.ids $O/ab.txt
