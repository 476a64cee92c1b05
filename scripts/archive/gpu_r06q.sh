#!/bin/bash
# round 6: stamps of the shipped instances at configs 1, 3, 5 (mb by shape) and 2 (16x16x4)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=${1:-r06q}
PKG=non-iid-distributed-learning-with-optimal-mixture-weights_amd
mkdir -p gpurun_out/$R
S=gpurun_out/$R/stamps.txt
L=$PWD/$PKG/libfedsim_stamps.so
FEDSIM_LIB=$L timeout -k 10 120 python -u scripts/stamps.py --config 1 >> $S 2>&1 || exit 1; echo "^ c1 (mb)" >> $S
FEDSIM_LIB=$L timeout -k 10 120 python -u scripts/stamps.py --config 3 --prox >> $S 2>&1 || exit 1; echo "^ c3 (mb)" >> $S
FEDSIM_LIB=$L timeout -k 10 120 python -u scripts/stamps.py --config 5 >> $S 2>&1 || exit 1; echo "^ c5 (mb)" >> $S
FEDSIM_LIB=$L timeout -k 10 120 python -u scripts/stamps.py --config 2 >> $S 2>&1 || exit 1; echo "^ c2 (16x16x4)" >> $S
grep -v amdgpu.ids $S
