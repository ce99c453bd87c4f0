# Ritz-apply variants (CAL_APPLY_1W 0/1) on the diagnostics-only run, with
# kernel stats, then the diagnostics parity subset under the variant
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-apply_ab}
mkdir -p $O
export TMPDIR=/tmp
for v in ${VALS:-0 1}; do
  ( cd /tmp && env "${VAR:-CAL_APPLY_1W}=$v" DIAG_REPS=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o run -- \
      python3 $GRAFT_REPO_ROOT/tools/diag_only.py > $O/diag_$v.json 2> $O/diag_$v.err ) || exit $?
  echo "1w=$v $(cat $O/diag_$v.json)"
  python3 - "$O/prof_$v/run_kernel_stats.csv" <<'PY'
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'apply_mt' in r['Name']: print('   ', r['Name'][:34], r['Calls'], round(float(r['AverageNs'])/1e3,1))
PY
done
env ${TESTENV:-CAL_APPLY_1W=1} timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py -x -q -m gpu -k "ritz or diag or rnorm or fullsize or harness or orth_err" --timeout 500 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; exit $rc
