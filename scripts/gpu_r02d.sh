#!/bin/bash
# Round 2, fourth GPU pass: multi-rank tests (sharded Z-GEMM FedAMW over 2 gloo ranks), bench
# lines (config 2 with the FedAMW leg; configs 3, 4, 5), kernel-trace stats, PMC passes.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r02d
mkdir -p $OUT
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -v --timeout 200 --timeout-method thread \
  > $OUT/dist.log 2>&1; rc=$?; echo "dist rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" $OUT/dist.log | tail; ok $rc || exit $rc
timeout -k 10 300 python -u bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err; rc=$?; echo "bench c2 rc=$rc"; cat $OUT/bench_c2.json; [ $rc -eq 0 ] || exit $rc
for c in 3 4 5; do
  timeout -k 10 300 python -u bench.py --config $c --steps 5 --warmup 2 --cpu-seconds 5 > $OUT/bench_c$c.json 2> $OUT/bench_c$c.err
  rc=$?; echo "bench c$c rc=$rc"; cat $OUT/bench_c$c.json; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 -u bench.py --no-cpu-baseline \
  > $OUT/kt.log 2>&1; rc=$?; echo "kernel trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash scripts/pmc_capture.sh c2 "--steps 3 --warmup 1 --no-fedamw-leg" "local_train" || exit 1
bash scripts/pmc_capture.sh c5 "--config 5 --steps 2 --warmup 1" "local_train|mix_solve|mix_z" || exit 1
bash scripts/pmc_capture.sh c2_fedamw "--algo fedamw --steps 2 --warmup 1" "mix_solve|mix_z" || exit 1
bash scripts/pmc_capture.sh c3 "--config 3 --steps 2 --warmup 1" "local_train" || exit 1
exit 0
