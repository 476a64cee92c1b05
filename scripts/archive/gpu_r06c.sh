#!/bin/bash
# round 6: the double-buffered split instance -- its tests, then launch times against the split form
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=${1:-r06c}
mkdir -p gpurun_out/$R
timeout -k 10 400 python -u -m pytest tests/test_gpu_dbuf.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/$R/dbuf_tests.log 2>&1; rc=$?
tail -3 gpurun_out/$R/dbuf_tests.log
grep -E "FAILED|Error" gpurun_out/$R/dbuf_tests.log | head -10
[ $rc -eq 0 ] || { echo "dbuf tests rc=$rc"; exit 1; }
S=gpurun_out/$R/lt.txt
for k in 1 2; do
  for d in off on; do
    timeout -k 10 120 python -u scripts/lt_sweep.py --config 2 --reg 0 --reps 30 --dbuf $d >> $S 2>&1 || exit 1; echo "^ c2 dbuf $d" >> $S
    timeout -k 10 120 python -u scripts/lt_sweep.py --config 5 --reg 1 --reps 10 --dbuf $d >> $S 2>&1 || exit 1; echo "^ c5 dbuf $d" >> $S
    timeout -k 10 120 python -u scripts/lt_sweep.py --config 1 --reg 1 --reps 10 --dbuf $d >> $S 2>&1 || exit 1; echo "^ c1 dbuf $d" >> $S
    timeout -k 10 120 python -u scripts/lt_sweep.py --config 4 --G 2 --reg 0 --reps 30 --dbuf $d >> $S 2>&1 || exit 1; echo "^ c4 G2 dbuf $d" >> $S
  done
done
grep -v amdgpu.ids $S
