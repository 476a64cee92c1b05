#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r02s2qmc2}; mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
FS_MIX_QMC_NK=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "qmc" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; echo "tests nk4 rc=$?"
grep -E "passed|failed" $O/tests.log | tail -2
for cfg in "8 12" "8 16" "4 8" "4 12" "4 16" "8 12" ; do set -- $cfg
  FS_MIX_QMC_NK=$1 FS_MIX_SOLVER=qmc FS_MIX_PF_H=$2 step "nk $1 h $2" timeout -k 10 150 python -u scripts/mix_time.py 1000 10 32000 2 >> $O/time.log 2>&1
  tail -2 $O/time.log | head -1 | sed 's/.*mix_solve//'
done
