# Round profile: kernel-trace stats of the bench + separate PMC passes (one counter group each).
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
TAG=${1:-r01}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof_$TAG -o $TAG --output-format csv -- python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1
echo "trace rc=$?"
OUT=gpurun_out/pmc
rm -rf $OUT; mkdir -p $OUT
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU" "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-include-regex "local_train|eval_kernel|aggregate_kernel" -d $OUT/p$i -o p$i --output-format csv -- python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/p$i.log 2>&1
  echo "pass $i ($grp) rc=$?"
done
