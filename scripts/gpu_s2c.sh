#!/bin/bash
# p-solve bound probe: config-2 shape with Z at full size (51 MB, Infinity Cache) vs a Z that
# fits one XCD's L2 (n_val 512: 2 MB), plain and with the s_memtime phase-stamp build.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02s2c; mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
for a in "100 10 12800 10" "100 10 512 250" "100 10 2048 64" "100 10 128 1000"; do
  FS_MIX_SOLVER=reg step "plain $a" timeout -k 10 120 python -u scripts/mix_time.py $a >> $O/time.log 2>&1
  FS_MIX_SOLVER=reg FEDSIM_LIB=$PWD/non-iid-distributed-learning-with-optimal-mixture-weights_amd/libfedsim_stamps.so step "stamps $a" timeout -k 10 120 python -u scripts/mix_time.py $a >> $O/time.log 2>&1
done
grep -E 'mix_solve|ticks' $O/time.log
