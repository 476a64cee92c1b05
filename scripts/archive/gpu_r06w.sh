#!/bin/bash
# round 6 (session 2): config 2's width on 4-wave workgroups of 4 tiles per wave (diagnostic
# build wide4.so, -DSP_WIDE4=1) against the shipped 8-wave instances, launch us (lt_sweep)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
PKG=non-iid-distributed-learning-with-optimal-mixture-weights_amd
O=gpurun_out/r06w; mkdir -p $O
for k in 1 2; do
  for lib in libfedsim wide4; do
    for mb in off on; do
      FEDSIM_LIB=$PKG/$lib.so timeout -k 10 120 python -u scripts/lt_sweep.py --config 2 --G 2 --reg 0 --mb $mb >> $O/ab.txt 2>&1 || exit 1
      echo "^ c2 $lib mb $mb" >> $O/ab.txt
    done
  done
done
cat $O/ab.txt
