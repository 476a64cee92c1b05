#!/bin/bash
# Z-GEMM check on one box: the fs_mix_z shape tests, the Z-dependent parity tests, then timing at
# configs 5 and 2 (scripts/z_time.py), each step under its own limit.   scripts/gpu_z.sh <tag>
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-z}
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread \
  -k "mix_z or test_mix_solve_variants" > gpurun_out/$TAG/z_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/$TAG/z_tests.log; exit 1; }
tail -2 gpurun_out/$TAG/z_tests.log
timeout -k 10 120 python -u scripts/z_time.py 1000 10 16384 32000 5 > gpurun_out/$TAG/z_c5.txt 2>&1 || { echo "z c5 rc=$?"; cat gpurun_out/$TAG/z_c5.txt; exit 1; }
cat gpurun_out/$TAG/z_c5.txt
timeout -k 10 120 python -u scripts/z_time.py 100 10 2048 12800 10 > gpurun_out/$TAG/z_c2.txt 2>&1 || { echo "z c2 rc=$?"; cat gpurun_out/$TAG/z_c2.txt; exit 1; }
cat gpurun_out/$TAG/z_c2.txt
timeout -k 10 120 python -u scripts/z_time.py 125 10 16384 32000 5 > gpurun_out/$TAG/z_c5_8rank.txt 2>&1 || { echo "z c5/8 rc=$?"; cat gpurun_out/$TAG/z_c5_8rank.txt; exit 1; }
cat gpurun_out/$TAG/z_c5_8rank.txt
timeout -k 10 120 rocprofv3 -L > gpurun_out/$TAG/counters.txt 2>&1 || echo "rocprofv3 -L rc=$?"
grep -iE "MALL|DRAM|EA0_RD|EA_RD|TCC_EA" gpurun_out/$TAG/counters.txt | head -40
