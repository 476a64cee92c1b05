#!/bin/bash
# round 6 (session 2): the mb image's row stride 4 mod 32 (conflict-free image writes) -- the mb
# tests and the config tests, then launch us against the first form (rsp8.so, -DSP_MB_RSP=8)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
PKG=non-iid-distributed-learning-with-optimal-mixture-weights_amd
O=gpurun_out/r06x; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_mb.py tests/test_gpu_configs.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || exit $rc
for k in 1 2; do
  for lib in libfedsim rsp8; do
    FEDSIM_LIB=$PKG/$lib.so timeout -k 10 120 python -u scripts/lt_sweep.py --config 3 --G 4 --prox >> $O/ab.txt 2>&1 || exit 1
    FEDSIM_LIB=$PKG/$lib.so timeout -k 10 120 python -u scripts/lt_sweep.py --config 5 --G 16 >> $O/ab.txt 2>&1 || exit 1
    FEDSIM_LIB=$PKG/$lib.so timeout -k 10 120 python -u scripts/lt_sweep.py --config 1 --G 8 >> $O/ab.txt 2>&1 || exit 1
    echo "^ $lib" >> $O/ab.txt
  done
done
grep -v amdgpu.ids $O/ab.txt
