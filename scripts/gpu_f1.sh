# Single-shot algorithms + feature map: GPU parity tests and feature-map timing.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/f1; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_single.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -20 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u scripts/fm_time.py > $O/fm_time.log 2>&1
rc=$?; echo "fm_time rc=$rc"; cat $O/fm_time.log; exit $rc
