#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r02s2ev2}; mkdir -p $O
for wv in 8 4; do
  FS_EVAL_WAVES=$wv timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "eval or golden" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/t$wv.log 2>&1; echo "waves $wv tests rc=$? $(tail -1 $O/t$wv.log)"
  FS_EVAL_WAVES=$wv timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p$wv -o p --output-format csv -- python3 -u bench.py --steps 10 --warmup 2 --no-fedamw-leg --no-cpu-baseline > $O/p$wv.log 2>&1; echo "c2 prof rc=$?"
  FS_EVAL_WAVES=$wv timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/q$wv -o q --output-format csv -- python3 -u bench.py --config 3 --steps 2 --warmup 1 --no-cpu-baseline > $O/q$wv.log 2>&1; echo "c3 prof rc=$?"
  for x in p q; do python3 -c "
import csv
for row in csv.reader(open('$O/$x$wv/${x}_kernel_stats.csv')):
    if 'eval_kernel' in row[0]: print('$x waves $wv', row[1], '%.1f us' % (float(row[3])/1e3))"; done
done
