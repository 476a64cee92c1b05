#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r02s2aa}; mkdir -p $O
for cfg in "default" "flags0" "noev" "default"; do
  case $cfg in default) E="X=1";; flags0) E="FS_TIMER_FLAGS=0";; noev) E="FS_BENCH_NO_EVENTS=1";; esac
  env $E FS_BENCH_HOST_TIMES=1 timeout -k 10 300 python -u bench.py --steps 100 --no-fedamw-leg --no-cpu-baseline > $O/b_$cfg.json 2> $O/b_$cfg.err
  echo "$cfg rc=$? $(grep 'host us' $O/b_$cfg.err) $(python3 -c "import json; print('launch_ms', json.loads(open('$O/b_$cfg.json').readline())['roofline']['launch_ms'])")"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o c2 --output-format csv -- python3 -u bench.py --steps 30 --warmup 2 --no-fedamw-leg --no-cpu-baseline > $O/prof.log 2>&1; echo "prof rc=$?"
grep local_train $O/prof/c2_kernel_stats.csv | cut -d, -f1-4 | cut -c1-200
tail -1 $O/prof.log | python3 -c "import json,sys; print('prof-run launch_ms', json.loads(sys.stdin.read())['roofline']['launch_ms'])"
