#!/bin/bash
# the whole GPU suite and smoke() (the driver's round-end checks) into gpurun_out/<tag>/
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=${1:-r06_suite}
mkdir -p gpurun_out/$R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$R/tests.log 2>&1
rc=$?
tail -3 gpurun_out/$R/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$R/smoke.log 2>&1 || { tail -20 gpurun_out/$R/smoke.log; exit 1; }
tail -2 gpurun_out/$R/smoke.log
