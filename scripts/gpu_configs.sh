# Bench lines + kernel stats for the other single-GPU configs (config 3 FedProx, config 2 FedAMW)
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
C3="--algo fedprox --clients 1000 --rows 465 --D 4096 --C 7 --test 50000 --shape covtype"
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline $C3 > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err
rc=$?; echo "bench c3 rc=$rc"; cat gpurun_out/bench_c3.json; tail -3 gpurun_out/bench_c3.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --algo fedamw > gpurun_out/bench_amw.json 2> gpurun_out/bench_amw.err
rc=$?; echo "bench amw rc=$rc"; cat gpurun_out/bench_amw.json; tail -3 gpurun_out/bench_amw.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o c3 --output-format csv -- python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline $C3 > gpurun_out/prof_c3.log 2>&1
rc=$?; echo "prof c3 rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_amw -o amw --output-format csv -- python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --algo fedamw > gpurun_out/prof_amw.log 2>&1
rc=$?; echo "prof amw rc=$rc"
exit $rc
