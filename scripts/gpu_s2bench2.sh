#!/bin/bash
# Bench lines at configs 2 (default, + CPU baseline) and 4 on the committed sources
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-s2bench2}; mkdir -p $O
timeout -k 10 300 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err && \
timeout -k 10 300 python -u bench.py --config 4 > $O/bench_c4.json 2> $O/bench_c4.err
