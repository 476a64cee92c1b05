#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r02s2r}; mkdir -p $O
timeout -k 10 200 python -u scripts/host_calls.py > $O/host_calls.log 2>&1; echo "rc=$?"; cat $O/host_calls.log | grep -v amdgpu.ids
