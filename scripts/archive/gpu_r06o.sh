#!/bin/bash
# round 6: mb softmax on NCS lanes per row -- tests, then configs 1 / 3 / 5
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=${1:-r06o}
mkdir -p gpurun_out/$R
timeout -k 10 600 python -u -m pytest tests/test_gpu_mb.py tests/test_gpu_split_early.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$R/tests.log 2>&1
rc=$?
tail -3 gpurun_out/$R/tests.log
[ $rc -eq 0 ] || exit $rc
S=gpurun_out/$R/lt.txt
for k in 1 2; do
  timeout -k 10 120 python -u scripts/lt_sweep.py --config 1 --reg 1 --reps 10 >> $S 2>&1 || exit 1; echo "^ c1 auto" >> $S
  timeout -k 10 120 python -u scripts/lt_sweep.py --config 3 --reg 0 --prox --reps 5 >> $S 2>&1 || exit 1; echo "^ c3 auto" >> $S
  timeout -k 10 120 python -u scripts/lt_sweep.py --config 5 --reg 1 --reps 10 >> $S 2>&1 || exit 1; echo "^ c5 auto" >> $S
done
grep -v amdgpu.ids $S
