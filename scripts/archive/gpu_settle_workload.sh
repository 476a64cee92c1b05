#!/bin/bash
# A/B of the bench's device settle: the workload's own training launches (default) vs GEMM+copy
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/settlew
mkdir -p $O
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/work_full.json 2> $O/work_full.err || { echo "bench rc=$?"; tail -30 $O/work_full.err; exit 1; }
cut -c1-400 $O/work_full.json
for k in 1 2; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/work_$k.json 2> $O/work_$k.err || { echo "bench rc=$?"; tail -30 $O/work_$k.err; exit 1; }
  FS_BENCH_SETTLE_KIND=mixed timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/mixed_$k.json 2> $O/mixed_$k.err || { echo "bench rc=$?"; tail -30 $O/mixed_$k.err; exit 1; }
done
python - <<'P'
import json,glob
for f in sorted(glob.glob('gpurun_out/settlew/*.json')):
    d=json.load(open(f))
    s='%-28s c2 %.0f %.4f ms frac %.4f' % (f.split('/')[-1], d['value'], d['ms_per_step'], d['roofline']['frac'])
    for c in ('config3','config4','config5'):
        if c in d: s+=' | %s %.0f frac %.4f' % (c, d[c]['value'], d[c]['roofline']['frac'])
    print(s)
P
