#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r02s2pk}; mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step tests timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "quad or prefetch or auto_choice or fedamw or golden" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
tail -1 $O/tests.log
for a in "100 10 12800 10" "64 7 12800 10" "128 10 12800 10" "10 5 2048 50"; do
  FS_MIX_SOLVER=quad step "quad $a" timeout -k 10 120 python -u scripts/mix_time.py $a >> $O/time.log 2>&1
  tail -2 $O/time.log | head -1
done
