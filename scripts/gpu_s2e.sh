#!/bin/bash
# quarter-wave p-solver: parity tests, then timing vs the register solver (+ helpers)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r02s2e}; mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step tests timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "quad or prefetch" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
tail -2 $O/tests.log
for cfg in "quad 0 100 10 12800 10" "quad 3 100 10 12800 10" "quad 6 100 10 12800 10" "quad 0 100 10 512 250" "reg 0 100 10 12800 10" "quad 0 64 7 12800 10" "quad 3 64 7 12800 10" "quad 0 10 2 2048 50" "wave 0 10 2 2048 50"; do set -- $cfg
  FS_MIX_SOLVER=$1 FS_MIX_PF_H=$2 step "$cfg" timeout -k 10 120 python -u scripts/mix_time.py $3 $4 $5 $6 >> $O/time.log 2>&1
  tail -2 $O/time.log | head -1
done
