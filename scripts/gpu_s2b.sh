#!/bin/bash
# Session-2 check: full GPU suite + smoke + bench c2 + rocprof stats, then the p-solve L2
# prefetch-helper sweep at config 2 (FS_MIX_PF_H helpers, FS_MIX_PF_LEAD steps ahead).
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r02s2b}
O=gpurun_out/$TAG
mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step pf_tests timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "prefetch or mix_solve_variants or auto_choice" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pf_tests.log 2>&1
tail -2 $O/pf_tests.log
for hl in "0 16" "1 16" "2 16" "3 16" "4 16" "6 16" "3 8" "3 32" "4 48"; do set -- $hl
  FS_MIX_SOLVER=reg FS_MIX_PF_H=$1 FS_MIX_PF_LEAD=$2 step "mix_time h=$1 lead=$2" timeout -k 10 120 python -u scripts/mix_time.py 100 10 12800 10 >> $O/pf_sweep.log 2>&1
  tail -2 $O/pf_sweep.log | head -1
done
step pytest timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
tail -2 $O/gpu_tests.log
step smoke timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
step bench_c2 timeout -k 10 300 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err
cat $O/bench_c2.json
