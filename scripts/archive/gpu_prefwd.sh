#!/bin/bash
# round 5 session 2: the split form with tile 0's forward at the end of the previous step
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/prefwd
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_split_early.py tests/test_gpu_pair.py tests/test_gpu_teams.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for c in 2 5; do
  timeout -k 10 200 python -u scripts/lt_sweep.py --config $c --reg 0 >> $O/lt.txt 2>&1 || { echo "sweep rc=$?"; tail -20 $O/lt.txt; exit 1; }
done
timeout -k 10 200 python -u scripts/lt_sweep.py --config 3 --prox --reg 0 >> $O/lt.txt 2>&1 || { echo "sweep rc=$?"; tail -20 $O/lt.txt; exit 1; }
timeout -k 10 200 python -u scripts/lt_sweep.py --config 1 --G 8 >> $O/lt.txt 2>&1 || { echo "sweep rc=$?"; tail -20 $O/lt.txt; exit 1; }
grep -v amdgpu.ids $O/lt.txt
for k in 1 2; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_$k.json 2> $O/bench_$k.err || { echo "bench rc=$?"; tail -30 $O/bench_$k.err; exit 1; }
done
python - <<'P'
import json,glob
for f in sorted(glob.glob('gpurun_out/prefwd/bench_*.json')):
    d=json.load(open(f))
    s='%-14s c2 %.0f %.4f ms launch %.4f frac %.4f' % (f.split('/')[-1], d['value'], d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac'])
    for c in ('config1','config3','config4','config5'):
        if c in d: s+=' | %s %.0f frac %s' % (c, d[c]['value'], ('%.4f' % d[c]['roofline']['frac']) if 'roofline' in d[c] else '-')
    print(s)
P
