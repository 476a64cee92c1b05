#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r02s2qmc}; mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "qmc" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; echo "tests rc=$?"
grep -E "passed|failed|Error" $O/tests.log | tail -5
for cfg in "qmc 0" "qmc 8" "qmc 16" "qmc 24" "mc 0"; do set -- $cfg
  FS_MIX_SOLVER=$1 FS_MIX_PF_H=$2 step "$cfg" timeout -k 10 150 python -u scripts/mix_time.py 1000 10 32000 1 >> $O/time.log 2>&1
  tail -2 $O/time.log | head -1 | sed 's/.*mix_solve//'
done
FS_MIX_SOLVER=qmc FS_MIX_PF_H=16 step "qmc 300" timeout -k 10 150 python -u scripts/mix_time.py 300 4 12800 2 >> $O/time.log 2>&1; tail -2 $O/time.log | head -1 | sed 's/.*mix_solve//'
FS_MIX_SOLVER=mc step "mc 300" timeout -k 10 150 python -u scripts/mix_time.py 300 4 12800 2 >> $O/time.log 2>&1; tail -2 $O/time.log | head -1 | sed 's/.*mix_solve//'
