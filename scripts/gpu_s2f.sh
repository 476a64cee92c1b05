#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r02s2f}; mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
timeout -k 10 60 ./scripts/probe/quad_lanes > $O/probe.log 2>&1; echo "probe rc=$?"; tail -45 $O/probe.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "quad" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; echo "tests rc=$?"
grep -E 'passed|failed|Error:' $O/tests.log | head -20
FS_MIX_SOLVER=quad step "time quad" timeout -k 10 120 python -u scripts/mix_time.py 100 10 12800 10 >> $O/time.log 2>&1
FS_MIX_SOLVER=quad FS_MIX_PF_H=4 step "time quad pf4" timeout -k 10 120 python -u scripts/mix_time.py 100 10 12800 10 >> $O/time.log 2>&1
grep mix_solve $O/time.log
