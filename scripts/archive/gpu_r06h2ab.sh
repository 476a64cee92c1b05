cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06h2; mkdir -p $O; rm -f $O/ab.txt
for k in 1 2 3 4; do
  for mb in auto off on; do
    timeout -k 10 120 python -u scripts/lt_sweep.py --config 2 --G 2 --reg 0 --mb $mb --reps 30 >> $O/ab.txt 2>&1 || exit 1
    echo "^ c2 mb $mb" >> $O/ab.txt
  done
done
grep -v amdgpu.ids $O/ab.txt
