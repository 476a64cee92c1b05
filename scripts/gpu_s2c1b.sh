#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r02s2c1b}; mkdir -p $O
for a in "10 2" "16 4" "5 3" "12 4"; do for sv in wave quad; do set -- $a
  FS_MIX_SOLVER=$sv timeout -k 10 150 python -u scripts/mix_time.py $1 $2 6512 20 >> $O/time.log 2>&1; echo "$a $sv rc=$? $(tail -2 $O/time.log | head -1 | sed 's/.*mix_solve//')"
done; done
