# Round 5: TSQR / parity subset after the fold changes, then the MFMA counters.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r05_check}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_tsqr.py tests/test_gpu_parity.py -x -q -m gpu -k "${PK:-tsqr or fold or project or lanczos}" --timeout 600 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
TAG=r05_pmc_mfma bash tools/gpu_r05_pmc_mfma.sh
