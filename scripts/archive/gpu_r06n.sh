#!/bin/bash
# round 6: the whole GPU suite and smoke on the mb-by-shape library, then the default bench line
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=${1:-r06n}
mkdir -p gpurun_out/$R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$R/tests.log 2>&1
rc=$?
tail -3 gpurun_out/$R/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$R/smoke.log 2>&1 || { tail -20 gpurun_out/$R/smoke.log; exit 1; }
tail -2 gpurun_out/$R/smoke.log
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/$R/bench.json 2> gpurun_out/$R/bench.err \
    || { echo "bench rc=$?"; tail -30 gpurun_out/$R/bench.err; exit 1; }
cut -c1-300 gpurun_out/$R/bench.json
