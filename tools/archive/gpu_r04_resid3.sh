# Round 4: residual probe (tools/resid_probe.hip) and the library's residual shape sweep with
# one Ritz pair per block (CAL_RESID_SHAPE=1xP), lane-shared slots off/on.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r04_resid3}
mkdir -p $O
timeout -k 10 300 ./tools/resid_probe 32 > $O/probe.txt 2>&1 || exit $?
cat $O/probe.txt
for v in ${COMBOS:-1x2 1x4 1x8 2x4 4x4}; do
  for L in 0 1; do
    CAL_RESID_LANE=$L CAL_RESID_SHAPE=$v DIAG_REPS=2 timeout -k 10 300 python tools/diag_only.py > $O/diag_${v}_l$L.json 2> $O/diag_${v}_l$L.err || exit $?
    echo "shape=$v lane=$L $(cat $O/diag_${v}_l$L.json)"
  done
done
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_tsqr.py tests/test_abi.py -x -v -m gpu -k "complex_pair or test_hooks or declined or fused" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
exit $rc
