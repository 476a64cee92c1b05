#!/bin/bash
# round 6 (session 2): config 2 (G = 2) early-issue depth with the mb and 16x16x4 instances
# (variant builds e8 / e12 / e16: -DSP_E1=d -DSP_G2_EARLY=d), launch us (lt_sweep)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
PKG=non-iid-distributed-learning-with-optimal-mixture-weights_amd
O=gpurun_out/r06e2; mkdir -p $O
for k in 1 2; do
  for lib in libfedsim e8 e12 e16; do
    for mb in off on; do
      FEDSIM_LIB=$PKG/$lib.so timeout -k 10 120 python -u scripts/lt_sweep.py --config 2 --G 2 --reg 0 --mb $mb >> $O/ab.txt 2>&1 || exit 1
      echo "^ c2 $lib mb $mb" >> $O/ab.txt
    done
  done
done
grep -v amdgpu.ids $O/ab.txt
