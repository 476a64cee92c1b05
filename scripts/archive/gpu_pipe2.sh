cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pipe2
timeout -k 10 300 python -u scripts/pipe_debug.py > gpurun_out/pipe2/debug.txt 2>&1; echo "debug rc=$?"; cat gpurun_out/pipe2/debug.txt | grep -v amdgpu.ids
timeout -k 10 300 python -u scripts/lt_time.py 100 2 1026 2 1026 > gpurun_out/pipe2/lt_time.txt 2>&1 || { echo "lt rc=$?"; tail gpurun_out/pipe2/lt_time.txt; exit 1; }
cat gpurun_out/pipe2/lt_time.txt
for f in pipe auto; do
  timeout -k 10 300 python -u bench.py --no-legs --no-cpu-baseline --train-form $f > gpurun_out/pipe2/bench_$f.json 2> gpurun_out/pipe2/bench_$f.err || { echo "bench rc=$?"; tail -30 gpurun_out/pipe2/bench_$f.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/pipe2/bench_$f.json')); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], r['frac'], r['launch_ms'], r['form'])"
done
