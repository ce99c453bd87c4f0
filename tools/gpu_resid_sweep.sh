# Same-box sweep of the batched residual kernel's shape (Ritz pairs per block
# CAL_RESID_CPB x row pairs per thread CAL_RESID_PPT) on the diagnostics-only
# run (tools/diag_only.py, lap3d_215, 15 iterations)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-resid_sweep}
mkdir -p $O
for v in ${COMBOS:-4x4 2x4 2x8 1x8 4x2 2x2 4x4}; do
  set -- ${v/x/ }
  CAL_RESID_CPB=$1 CAL_RESID_PPT=$2 DIAG_REPS=2 timeout -k 10 300 python tools/diag_only.py > $O/diag_c$1_p$2.json 2> $O/diag_c$1_p$2.err || exit $?
  echo "cpb=$1 ppt=$2 $(cat $O/diag_c$1_p$2.json)"
done
