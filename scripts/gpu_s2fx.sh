#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r02s2fx}; mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
FS_MIX_QUAD_FASTEXP=1 step tests timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "quad or fedamw or golden" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
grep -E "passed|failed" $O/tests.log | tail -1
for fx in 0 1 0 1; do
  FS_MIX_QUAD_FASTEXP=$fx FS_MIX_SOLVER=quad step "fastexp $fx" timeout -k 10 120 python -u scripts/mix_time.py 100 10 12800 10 >> $O/time.log 2>&1
  tail -2 $O/time.log | head -1 | sed 's/.*mix_solve//'
done
