set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/exp; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_experiment.py tests/test_gpu_single.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|error" $O/tests.log | tail -30; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u run_experiment.py --dataset a9a --D 2000 --clients 10 --rounds 100 --quiet --result-dir gpurun_out/exp > $O/exp_a9a.log 2>&1
rc=$?; echo "exp rc=$rc"; tail -12 $O/exp_a9a.log; exit $rc
