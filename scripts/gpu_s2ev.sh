#!/bin/bash
# eval row tiles per workgroup: unit golden test + kernel time at configs 2 and 3
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r02s2ev}; mkdir -p $O
for r in 1 2 4; do
  FS_EVAL_RTW=$r timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "eval or golden" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/t$r.log 2>&1; echo "rtw $r tests rc=$? $(tail -1 $O/t$r.log)"
  FS_EVAL_RTW=$r timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p$r -o p --output-format csv -- python3 -u bench.py --steps 10 --warmup 2 --no-fedamw-leg --no-cpu-baseline > $O/p$r.log 2>&1; echo "c2 prof rc=$?"
  grep eval_kernel $O/p$r/p_kernel_stats.csv | cut -d, -f2-4
  FS_EVAL_RTW=$r timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/q$r -o q --output-format csv -- python3 -u bench.py --config 3 --steps 2 --warmup 1 --no-cpu-baseline > $O/q$r.log 2>&1; echo "c3 prof rc=$?"
  grep eval_kernel $O/q$r/q_kernel_stats.csv | cut -d, -f2-4
done
