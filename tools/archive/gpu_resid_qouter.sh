set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/resid_q; mkdir -p $O
for v in "0 4 4" "1 4 4" "1 4 8" "1 8 4" "0 4 4" "1 4 4"; do
  set -- $v
  r=$(CAL_RESID_QOUTER=$1 CAL_RESID_CPB=$2 CAL_RESID_PPT=$3 DIAG_REPS=2 timeout -k 10 300 python tools/diag_only.py) || exit $?
  echo "qouter=$1 cpb=$2 ppt=$3 $r"
done
cd /tmp
CAL_RESID_QOUTER=1 DIAG_REPS=0 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "resid_multi" --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc_q1 -o run -- python3 $GRAFT_REPO_ROOT/tools/diag_only.py > $GRAFT_REPO_ROOT/$O/pmc_q1.log 2>&1
echo pmc rc=$?
