#!/bin/bash
# host API timeline vs kernel timeline at config 2 (where do the per-round gaps come from)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r02s2o}; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace -d $O/trace -o tr --output-format csv -- python3 -u bench.py --steps 10 --warmup 2 --no-fedamw-leg --no-cpu-baseline > $O/trace.log 2>&1
echo "trace rc=$?"
ls $O/trace
