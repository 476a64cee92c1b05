#!/bin/bash
# round 6 (session 2): fs_aggregate's one-launch form with every load of 8 clients issued before
# the first fold -- the parity and config tests, then the bench's aggregate timing (20 launches
# back to back) at configs 2, 3, 4 against the previous build (base.so), interleaved
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
PKG=non-iid-distributed-learning-with-optimal-mixture-weights_amd
O=gpurun_out/r06ag; mkdir -p $O; rm -f $O/ab.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || exit $rc
for k in 1 2 3; do
  for lib in libfedsim base; do
    FEDSIM_LIB=$PKG/$lib.so timeout -k 10 200 python -u bench.py --config 2 --no-legs --no-fedamw-leg --no-cpu-baseline --steps 20 --warmup 5 > $O/b.json 2>/dev/null || exit 1
    python -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('$lib', round(d['aggregate']['ms']*1e3,2), 'us', round(d['aggregate']['achieved']), 'GB/s', round(d['ms_per_step']*1e3,1), 'us/round')" >> $O/ab.txt
  done
done
cat $O/ab.txt
