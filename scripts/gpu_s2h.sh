#!/bin/bash
# quad p-solver: where a step's time goes (stamps), L2-resident Z vs full Z, helpers
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r02s2h}; mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
SL=$PWD/non-iid-distributed-learning-with-optimal-mixture-weights_amd/libfedsim_stamps.so
for cfg in "0 100 10 12800 10" "0 100 10 512 250" "0 100 10 128 1000" "4 100 10 12800 10" "8 100 10 12800 10" "0 64 7 12800 10" "0 10 2 2048 50"; do set -- $cfg
  FS_MIX_SOLVER=quad FS_MIX_PF_H=$1 step "plain $cfg" timeout -k 10 120 python -u scripts/mix_time.py $2 $3 $4 $5 >> $O/time.log 2>&1
  FS_MIX_SOLVER=quad FS_MIX_PF_H=$1 FEDSIM_LIB=$SL step "stamps $cfg" timeout -k 10 120 python -u scripts/mix_time.py $2 $3 $4 $5 >> $O/time.log 2>&1
done
grep -E 'mix_solve|ticks' $O/time.log
