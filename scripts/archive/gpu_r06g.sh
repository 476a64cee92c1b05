#!/bin/bash
# round 6: the split form's 4x4x1 multi-block ("mb") instances -- tests, then launch A/B at configs 1-5
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=${1:-r06g}
mkdir -p gpurun_out/$R
timeout -k 10 600 python -u -m pytest tests/test_gpu_mb.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$R/tests.log 2>&1
rc=$?
tail -5 gpurun_out/$R/tests.log
[ $rc -eq 0 ] || exit $rc
S=gpurun_out/$R/lt.txt
for k in 1 2; do
  for mb in off on; do
    timeout -k 10 120 python -u scripts/lt_sweep.py --config 2 --reg 0 --reps 30 --mb $mb >> $S 2>&1 || exit 1; echo "^ c2 mb $mb" >> $S
    timeout -k 10 120 python -u scripts/lt_sweep.py --config 5 --reg 1 --reps 10 --mb $mb >> $S 2>&1 || exit 1; echo "^ c5 mb $mb" >> $S
    timeout -k 10 120 python -u scripts/lt_sweep.py --config 1 --reg 1 --reps 10 --mb $mb >> $S 2>&1 || exit 1; echo "^ c1 mb $mb" >> $S
    timeout -k 10 120 python -u scripts/lt_sweep.py --config 3 --reg 0 --prox --reps 5 --mb $mb >> $S 2>&1 || exit 1; echo "^ c3 mb $mb" >> $S
    timeout -k 10 120 python -u scripts/lt_sweep.py --config 4 --reg 0 --G 2,4 --reps 20 --mb $mb >> $S 2>&1 || exit 1; echo "^ c4 split G2/G4 mb $mb" >> $S
  done
done
grep -v amdgpu.ids $S
