# Round 4 same-box A/B: non-temporal stores of the Ritz vectors (k_apply_mt, CAL_APPLY_NT=1) on the diagnostics-on run.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r04_apply_nt}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fullsize.py \
    -k "fullsize_vs_omp and not tsqr" > $O/pytest_on.log 2>&1 || exit 1
for i in 1 2 3; do for v in 0 1; do
  if [ $v = 1 ]; then export CAL_APPLY_NT=1; else unset CAL_APPLY_NT; fi
  timeout -k 10 300 python tools/diag_only.py > $O/d_${v}_$i.txt 2>&1 || exit 1
  echo "NT=$v $(tail -1 $O/d_${v}_$i.txt)"
done; done
