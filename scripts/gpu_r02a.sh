#!/bin/bash
# Round 2, first GPU pass: parity suite (split-group kernel rewrite) + local-train G sweep.
# Each GPU step has its own time limit; a fault / abort / timeout (rc not 0 or 1) ends the script.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r02a
mkdir -p $OUT
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -v --timeout 120 --timeout-method thread \
  > $OUT/parity.log 2>&1; rc=$?; echo "parity rc=$rc"; tail -3 $OUT/parity.log; ok $rc || exit $rc
for c in 2 3 4 5; do
  timeout -k 10 180 python -u scripts/lt_sweep.py --config $c --G 0,1,2,4,8,16 > $OUT/sweep_c$c.log 2>&1
  rc=$?; echo "sweep c$c rc=$rc"; cat $OUT/sweep_c$c.log | grep -v Warn; ok $rc || exit $rc
done
timeout -k 10 180 python -u scripts/lt_sweep.py --config 1 --G 1,2,4,8,16 --reps 3 > $OUT/sweep_c1.log 2>&1
rc=$?; echo "sweep c1 rc=$rc"; cat $OUT/sweep_c1.log; ok $rc || exit $rc
timeout -k 10 180 python -u scripts/lt_sweep.py --config 3 --G 1,4,8 --prox > $OUT/sweep_c3p.log 2>&1
rc=$?; echo "sweep c3 prox rc=$rc"; cat $OUT/sweep_c3p.log; ok $rc || exit $rc
exit 0
