#!/bin/bash
# FedAMW shuffles behind the training kernel: parity + config 5 / config 2 bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r02m
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "fedamw or plan or golden or config or abi" > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --config 5 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_c5.json 2> $OUT/bench_c5.err; rc=$?
tail -1 $OUT/bench_c5.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5', d['value'], d['ms_per_step'], d['roofline']['launch_ms'], d['fedamw'])"; [ $rc -eq 0 ] || exit $rc
