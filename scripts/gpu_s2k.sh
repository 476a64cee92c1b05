#!/bin/bash
# quad p-solver: out-of-range padding chunks (no memory access) x issue split x helpers
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r02s2k}; mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
FS_MIX_QUAD_SPLIT=5 step "tests" timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "quad" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
tail -1 $O/tests.log
for cfg in "1 10 0" "1 5 0" "1 3 0" "1 5 4" "1 3 4" "1 5 2" "1 4 4" "0 5 4" "1 5 6"; do set -- $cfg
  FS_MIX_SOLVER=quad FS_MIX_QUAD_OOB=$1 FS_MIX_QUAD_SPLIT=$2 FS_MIX_PF_H=$3 step "oob $1 split $2 pf $3" timeout -k 10 120 python -u scripts/mix_time.py 100 10 12800 10 >> $O/time.log 2>&1
  tail -2 $O/time.log | head -1
done
