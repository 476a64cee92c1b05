#!/bin/bash
# Kernel trace (rocprofv3 --kernel-trace --stats) of the default bench command.   scripts/gpu_trace.sh <tag>
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=${1:-r04}
mkdir -p gpurun_out/trace_$R
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_$R -o $R --output-format csv -- python3 -u bench.py \
  > gpurun_out/trace_$R/bench.json 2> gpurun_out/trace_$R/bench.err
rc=$?
echo "trace rc=$rc"
find gpurun_out/trace_$R -name "*stats*"
exit $rc
