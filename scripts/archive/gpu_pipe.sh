#!/bin/bash
# pipe form: its GPU tests, then launch times split vs pipe at config 2, then the bench line
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=${1:-pipe}
mkdir -p gpurun_out/$R
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipe.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/$R/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/$R/tests.log; exit 1; }
tail -3 gpurun_out/$R/tests.log
timeout -k 10 300 python -u scripts/lt_time.py 100 2 1026 2 1026 > gpurun_out/$R/lt_time.txt 2>&1 \
  || { echo "lt_time rc=$?"; tail -20 gpurun_out/$R/lt_time.txt; exit 1; }
cat gpurun_out/$R/lt_time.txt
for f in pipe auto; do
  timeout -k 10 300 python -u bench.py --no-legs --no-cpu-baseline --train-form $f > gpurun_out/$R/bench_$f.json 2> gpurun_out/$R/bench_$f.err \
    || { echo "bench rc=$?"; tail -30 gpurun_out/$R/bench_$f.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/$R/bench_$f.json')); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], r['frac'], r['launch_ms'], r['form'])"
done
