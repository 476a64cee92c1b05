#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r02s2lead}; mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
for cfg in "2 16" "3 16" "4 16" "6 16" "3 8" "3 24" "16 16"; do set -- $cfg
  FS_MIX_SOLVER=qmc FS_MIX_PF_LEAD=$1 FS_MIX_PF_H=$2 step "lead $1 h $2" timeout -k 10 150 python -u scripts/mix_time.py 1000 10 32000 2 >> $O/time.log 2>&1
  tail -2 $O/time.log | head -1 | sed 's/.*mix_solve//'
done
