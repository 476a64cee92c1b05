#!/bin/bash
# round 5 session 2: the narrow chained instances (config 1) -- tests, widths, stamps
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/narrow
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_split_early.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python -u scripts/lt_sweep.py --config 1 --G 4,8,16 > $O/widths.txt 2>&1 || { echo "sweep rc=$?"; tail -20 $O/widths.txt; exit 1; }
timeout -k 10 200 python -u scripts/lt_sweep.py --config 1 --G 4,8,16 --early off >> $O/widths.txt 2>&1 || { echo "sweep rc=$?"; tail -20 $O/widths.txt; exit 1; }
grep -v amdgpu.ids $O/widths.txt
bash scripts/gpu_stamps.sh narrow "--config 1" "--config 1 --G 4" "--config 1 --G 16"
