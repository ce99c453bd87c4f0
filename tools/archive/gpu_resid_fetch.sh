# FETCH_SIZE (and WRITE_SIZE) of the batched residual kernel per shape
# (CAL_RESID_CPB x CAL_RESID_PPT), diagnostics-only run, one PMC pass each
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-resid_fetch}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for v in ${COMBOS:-4x4 1x8 2x4}; do
  set -- ${v/x/ }
  CAL_RESID_CPB=$1 CAL_RESID_PPT=$2 DIAG_REPS=0 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "resid_multi" \
      --output-format csv -d $O/c$1_p$2 -o run -- python3 $GRAFT_REPO_ROOT/tools/diag_only.py > $O/c$1_p$2.log 2>&1
  rc=$?
  echo "cpb=$1 ppt=$2 rc=$rc $(tail -1 $O/c$1_p$2.log | head -c 200)"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
