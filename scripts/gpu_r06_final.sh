#!/bin/bash
# round 6 final: the whole GPU suite, smoke, then the default bench line twice (the driver's command)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=${1:-r06_final2}
mkdir -p gpurun_out/$R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$R/tests.log 2>&1
rc=$?
tail -3 gpurun_out/$R/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$R/smoke.log 2>&1 || { tail -20 gpurun_out/$R/smoke.log; exit 1; }
tail -2 gpurun_out/$R/smoke.log
for k in a b; do
  timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/$R/bench_$k.json 2> gpurun_out/$R/bench_$k.err \
    || { echo "bench rc=$?"; tail -30 gpurun_out/$R/bench_$k.err; exit 1; }
  cut -c1-200 gpurun_out/$R/bench_$k.json
done
