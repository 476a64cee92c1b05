# Full GPU suite + bench lines (config 2 default with CPU baseline, config 3, config 2 FedAMW)
# + rocprofv3 kernel-trace stats of each.  Every GPU step under its own timeout, chained.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
TAG=${1:-r01b}
O=gpurun_out/$TAG
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step pytest timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
tail -3 $O/gpu_tests.log
step bench_c2 timeout -k 10 300 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err
cat $O/bench_c2.json
step bench_c3 timeout -k 10 300 python -u bench.py --config 3 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err
cat $O/bench_c3.json
step bench_amw timeout -k 10 300 python -u bench.py --algo fedamw --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_amw.json 2> $O/bench_amw.err
cat $O/bench_amw.json
step prof_c2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o c2 --output-format csv -- python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/prof_c2.log 2>&1
step prof_c3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o c3 --output-format csv -- python -u bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline > $O/prof_c3.log 2>&1
step prof_amw timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_amw -o amw --output-format csv -- python -u bench.py --algo fedamw --steps 3 --warmup 1 --no-cpu-baseline > $O/prof_amw.log 2>&1
