#!/bin/bash
# round 6 (session 2): config 1's chained width with the mb instances (launch us, lt_sweep)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06y; mkdir -p $O
for k in 1 2; do
  timeout -k 10 300 python -u scripts/lt_sweep.py --config 1 --G 2,4,8,16 >> $O/c1.txt 2>&1 || exit 1
done
grep -v amdgpu.ids $O/c1.txt
