#!/bin/bash
# Evidence for the current kernel sources: PMC passes (config 2 group kernel; config 2 FedAMW
# p-solve), rocprofv3 kernel-trace stats of the default bench, the default bench line.
#   scripts/gpu_s2cap.sh <tag> [configs...]   (configs: c2 c2_fedamw c3 c4 c5)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-s2}; shift
O=gpurun_out/$TAG; mkdir -p $O
[ $# -gt 0 ] || set -- c2 c2_fedamw
for c in "$@"; do
  case $c in
    c2) bash scripts/pmc_capture.sh c2 "--config 2 --steps 3 --warmup 1 --no-fedamw-leg" "local_train" || exit 1 ;;
    c2_fedamw) bash scripts/pmc_capture.sh c2_fedamw "--config 2 --algo fedamw --steps 1 --warmup 1" "mix_solve" || exit 1 ;;
    c3) bash scripts/pmc_capture.sh c3 "--config 3 --steps 2 --warmup 1" "local_train" || exit 1 ;;
    c4) bash scripts/pmc_capture.sh c4 "--config 4 --steps 3 --warmup 1" "local_train" || exit 1 ;;
    c5) bash scripts/pmc_capture.sh c5 "--config 5 --steps 1 --warmup 1" "local_train" || exit 1 ;;
  esac
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o c2 --output-format csv -- python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/prof_c2.log 2>&1
echo "prof_c2 rc=$?"
timeout -k 10 300 python3 -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err
echo "bench_c2 rc=$?"; cat $O/bench_c2.json
