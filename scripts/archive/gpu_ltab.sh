#!/bin/bash
# split local training A/B on one box: the current library vs libfedsim_prev.so (the same
# sources with the pre-team split kernel), configs 5 and 2, alternating
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-ltab}
mkdir -p gpurun_out/$TAG
OUT=gpurun_out/$TAG/ab.txt
: > $OUT
PKG=$PWD/non-iid-distributed-learning-with-optimal-mixture-weights_amd
for c in 5 2; do
  for lib in libfedsim_prev.so libfedsim.so libfedsim_prev.so libfedsim.so; do
    FEDSIM_LIB=$PKG/$lib timeout -k 10 200 python -u bench.py --config $c --no-legs --no-fedamw-leg --no-cpu-baseline \
      --steps 6 --warmup 2 > gpurun_out/$TAG/b.json 2> gpurun_out/$TAG/b.err || { echo "bench rc=$? c$c $lib"; tail -20 gpurun_out/$TAG/b.err; exit 1; }
    python -c "import json; d = json.loads(open('gpurun_out/$TAG/b.json').read().strip().splitlines()[-1]); r = d['roofline']; print('config $c $lib', round(d['ms_per_step'], 4), 'ms/round, launch', round(r['launch_ms'], 4), 'frac', round(r['frac'], 4), r['form'], r['group_width'])" >> $OUT
  done
done
cat $OUT
