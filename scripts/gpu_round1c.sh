# Full GPU suite + smoke + bench lines (config 2 default with CPU baseline, config 2 FedAMW,
# config 5 FedAMW with the multi-CU p-solve) + rocprofv3 kernel-trace stats of config 5.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
TAG=${1:-r01c}
O=gpurun_out/$TAG
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step pytest timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
tail -3 $O/gpu_tests.log
step smoke timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -2 $O/smoke.log
step bench_c2 timeout -k 10 300 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err
cat $O/bench_c2.json
step bench_amw timeout -k 10 300 python -u bench.py --algo fedamw --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_c2_fedamw.json 2> $O/bench_amw.err
cat $O/bench_c2_fedamw.json
step bench_c5 timeout -k 10 300 python -u bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err
cat $O/bench_c5.json
step prof_c5 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o c5 --output-format csv -- python -u bench.py --config 5 --steps 2 --warmup 1 --no-cpu-baseline > $O/prof_c5.log 2>&1
