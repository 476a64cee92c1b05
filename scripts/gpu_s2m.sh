#!/bin/bash
# multi-CU p-solver at config 5's shape with Infinity-Cache prefetch helpers (other XCDs)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r02s2m}; mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
FS_MIX_PF_H=16 step tests timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "multi_cu" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
tail -1 $O/tests.log
for cfg in "0 16 2" "16 16 2" "32 16 2" "64 16 2" "32 32 2" "32 8 2" "32 16 0" "32 16 1"; do set -- $cfg
  FS_MIX_SOLVER=mc FS_MIX_PF_H=$1 FS_MIX_PF_LEAD=$2 FS_MIX_MC_ZAT=$3 step "mc pf $1 lead $2 zat $3" timeout -k 10 150 python -u scripts/mix_time.py 1000 10 32000 1 >> $O/time.log 2>&1
  tail -2 $O/time.log | head -1
done
