#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r02s2c1}; mkdir -p $O
for cfg in "wave 0" "quad 0" "quad 4" "wave 0"; do set -- $cfg
  FS_MIX_SOLVER=$1 FS_MIX_PF_H=$2 timeout -k 10 150 python -u scripts/mix_time.py 10 2 6512 20 >> $O/time.log 2>&1; echo "$cfg rc=$?"
  tail -2 $O/time.log | head -1 | sed 's/.*mix_solve//'
done
for cfg in "wave 0" "quad 4"; do set -- $cfg
  FS_MIX_SOLVER=$1 FS_MIX_PF_H=$2 timeout -k 10 150 python -u scripts/mix_time.py 16 4 6512 20 >> $O/time.log 2>&1; echo "16x4 $cfg rc=$?"
  tail -2 $O/time.log | head -1 | sed 's/.*mix_solve//'
done
