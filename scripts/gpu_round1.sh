set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
echo "pytest rc=$?"; tail -5 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bench1.json 2> gpurun_out/bench1.err
echo "bench rc=$?"; cat gpurun_out/bench1.json; tail -3 gpurun_out/bench1.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof1 -o r01 --output-format csv -- python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof1.log 2>&1
echo "prof rc=$?"
