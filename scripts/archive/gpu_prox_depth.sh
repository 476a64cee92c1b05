#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
P=$PWD/non-iid-distributed-learning-with-optimal-mixture-weights_amd
for pass in 1 2; do
 for L in libfedsim.so libfedsim_proxearly1.so libfedsim_proxearly3.so libfedsim_proxearly4.so; do
  echo -n "$L pass $pass: "; FEDSIM_LIB=$P/$L timeout -k 10 150 python -u scripts/lt_sweep.py --config 3 --prox --reg 0 2>&1 | grep -v amdgpu.ids || exit 1
 done
done
