#!/bin/bash
# per-round overhead A/B at config 2: event release scope of the plan's ordering events, the
# per-round timing events of the bench, and a kernel trace of the default
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r02s2n}; mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
for cfg in "0 0" "1 0" "0 1" "1 1" "0 0"; do set -- $cfg
  FS_EVENT_FENCE=$1 FS_BENCH_NO_EVENTS=$2 step "fence $1 noev $2" timeout -k 10 200 python -u bench.py --steps 50 --warmup 3 --no-fedamw-leg --no-cpu-baseline > $O/b_$1_$2.json 2>$O/b.err
  python3 -c "import json; d=json.load(open('$O/b_$1_$2.json')); print('  ms/round %.4f launch_ms %s' % (d['ms_per_step'], d['roofline']['launch_ms']))"
done
step trace timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace -o tr --output-format csv -- python3 -u bench.py --steps 10 --warmup 2 --no-fedamw-leg --no-cpu-baseline > $O/trace.log 2>&1
