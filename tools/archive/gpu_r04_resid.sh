# Round 4: the rewritten batched residual kernel (k_resid_pairs): correctness on the
# diagnostics tests, then a same-box shape sweep (CAL_RESID_SHAPE = pairs-per-block x
# row-pairs-per-thread) on the diagnostics-only run and a rocprof kernel trace of it.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r04_resid}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -v -m gpu -k "${TESTK:-lanczos}" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
for v in ${COMBOS:-4x4 2x2 4x2 8x2 2x4 8x1 4x1}; do
  CAL_RESID_SHAPE=$v DIAG_REPS=2 timeout -k 10 300 python tools/diag_only.py > $O/diag_$v.json 2> $O/diag_$v.err || exit $?
  echo "shape=$v $(cat $O/diag_$v.json)"
done
cd /tmp && CAL_RESID_SHAPE=${PROF_SHAPE:-4x4} DIAG_REPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/diag_only.py > $O/prof.log 2>&1
echo "prof rc=$?"
