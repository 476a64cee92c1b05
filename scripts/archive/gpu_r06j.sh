#!/bin/bash
# round 6: the whole GPU suite on the mb-by-shape library, then launch times at configs 1-5 (mb by shape vs off)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=${1:-r06j}
mkdir -p gpurun_out/$R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$R/tests.log 2>&1
rc=$?
tail -3 gpurun_out/$R/tests.log
[ $rc -eq 0 ] || exit $rc
S=gpurun_out/$R/lt.txt
for k in 1 2; do
  for mb in auto off; do
    timeout -k 10 120 python -u scripts/lt_sweep.py --config 1 --reg 1 --reps 10 --mb $mb >> $S 2>&1 || exit 1; echo "^ c1 mb $mb" >> $S
    timeout -k 10 120 python -u scripts/lt_sweep.py --config 3 --reg 0 --prox --reps 5 --mb $mb >> $S 2>&1 || exit 1; echo "^ c3 mb $mb" >> $S
  done
done
grep -v amdgpu.ids $S
