#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r02s2t}; mkdir -p $O
FS_PLAN_TRACE=1 timeout -k 10 200 python -u scripts/host_calls.py > $O/host_calls.log 2>&1; echo "rc=$?"; grep -v amdgpu.ids $O/host_calls.log | tail -30
