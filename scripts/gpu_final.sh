# Round-end check of the committed tree: full GPU suite, smoke, default bench (+ CPU baseline),
# and the rocprofv3 kernel-trace summary of the default bench.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
TAG=${1:-r01d}
O=gpurun_out/$TAG
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step pytest timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
tail -2 $O/gpu_tests.log
step smoke timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
step bench_c2 timeout -k 10 300 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err
cat $O/bench_c2.json
step prof_c2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o c2 --output-format csv -- python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/prof_c2.log 2>&1
