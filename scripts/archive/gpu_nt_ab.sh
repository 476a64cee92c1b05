#!/bin/bash
# A/B: the split form's in-loop row loads nontemporal (diagnostic library libfedsim_nt.so) vs shipped
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
P=$PWD/non-iid-distributed-learning-with-optimal-mixture-weights_amd
for pass in 1 2; do
 for L in libfedsim.so libfedsim_nt.so; do
  for c in 2 5; do echo -n "$L pass $pass: "; FEDSIM_LIB=$P/$L timeout -k 10 120 python -u scripts/lt_sweep.py --config $c --reg 0 2>&1 | grep -v amdgpu.ids || exit 1; done
  echo -n "$L pass $pass: "; FEDSIM_LIB=$P/$L timeout -k 10 120 python -u scripts/lt_sweep.py --config 3 --prox --reg 0 2>&1 | grep -v amdgpu.ids || exit 1
 done
done
