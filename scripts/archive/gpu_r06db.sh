#!/bin/bash
# round 6 (session 2): config 2 on the double-buffered instance with the forward on the 4x4x1 MFMA
# (diagnostic build dbmbf.so, -DDB_MBF=1) vs the double-buffered 16x16x4 and the shipped split form
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
PKG=non-iid-distributed-learning-with-optimal-mixture-weights_amd
O=gpurun_out/r06db; mkdir -p $O; rm -f $O/ab.txt
for k in 1 2 3 4; do
  timeout -k 10 120 python -u scripts/lt_sweep.py --config 2 --G 2 --reg 0 --reps 30 >> $O/ab.txt 2>&1 || exit 1
  echo "^ split" >> $O/ab.txt
  timeout -k 10 120 python -u scripts/lt_sweep.py --config 2 --G 2 --reg 0 --reps 30 --dbuf on >> $O/ab.txt 2>&1 || exit 1
  echo "^ dbuf" >> $O/ab.txt
  FEDSIM_LIB=$PKG/dbmbf.so timeout -k 10 120 python -u scripts/lt_sweep.py --config 2 --G 2 --reg 0 --reps 30 --dbuf on >> $O/ab.txt 2>&1 || exit 1
  echo "^ dbuf mb-forward" >> $O/ab.txt
done
grep -v amdgpu.ids $O/ab.txt
