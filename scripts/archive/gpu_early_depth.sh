#!/bin/bash
# early-issue depth re-check after the pre-forward (round 5, session 2): shipped vs depth 2/6/8 (all widths)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
P=$PWD/non-iid-distributed-learning-with-optimal-mixture-weights_amd
for pass in 1 2; do
 for L in libfedsim.so libfedsim_plainearly2.so libfedsim_plainearly6.so libfedsim_plainearly8.so; do
  for c in 2 5; do
   echo -n "$L pass $pass: "; FEDSIM_LIB=$P/$L timeout -k 10 120 python -u scripts/lt_sweep.py --config $c --reg 0 2>&1 | grep -v amdgpu.ids || exit 1
  done
 done
done
