# Round 4 timing experiment: the residual probe kernel inside the library (CAL_RESID_PROBE=1)
# against the library's plane-march residual, diagnostics-only run, kernel stats of each.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r04_probe7}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for V in 0 1; do
  CAL_RESID_PROBE=$V DIAG_REPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof$V -o run -- python3 $GRAFT_REPO_ROOT/tools/diag_only.py > $O/prof$V.log 2>&1
  echo "probe=$V rc=$?"; tail -1 $O/prof$V.log
done
