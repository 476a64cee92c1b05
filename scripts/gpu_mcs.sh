# multi-CU p-solve: poll back-off sweep (s_sleep 0 / 2 / 8 between re-polls)
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
P=$PWD/non-iid-distributed-learning-with-optimal-mixture-weights_amd
T="timeout -k 10 120 python -u scripts/mix_time.py"
for lib in libfedsim_bo0.so libfedsim.so libfedsim_bo8.so; do
  echo "== $lib"
  FS_MIX_SOLVER=mc FEDSIM_LIB=$P/$lib $T 10 2 6500 2 && \
  FS_MIX_SOLVER=mc FEDSIM_LIB=$P/$lib $T 100 10 12800 2 && \
  FEDSIM_LIB=$P/$lib $T 1000 10 32000 1 || exit 1
done
