#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, each under a hard timeout) over one bench.py
# workload:  scripts/pmc_capture.sh <tag> "<bench.py args>" "<kernel regex>"
# Output: gpurun_out/pmc_<tag>/p<i>/...counter_collection.csv  (summarised by scripts/pmc_summary.py)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
# the bench's device settle as GEMMs / copies here: its default (the workload's training kernel,
# late-issue instance) would add settle launches to the captured kernels; counters are per launch,
# so the settle's kind changes nothing the capture reports
export FS_BENCH_SETTLE_KIND=mixed
TAG=$1; ARGS=$2; REGEX=$3
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
python3 -c "import sys, json; sys.path.insert(0, '.'); import fedamw_amd; from fedamw_amd import _lib; print(json.dumps({k: _lib.source_revision(k) for k in [None] + list(_lib.KERNEL_SOURCES)}))" \
  > $OUT/source_rev.json || exit 1
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS" \
  "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
  "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $grp --kernel-include-regex "$REGEX" -d $OUT/p$i -o p$i --output-format csv \
    -- python3 -u bench.py $ARGS --no-cpu-baseline > $OUT/p$i.log 2>&1
  rc=$?
  echo "pmc $TAG pass $i ($grp) rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
exit 0
