# Selected GPU test files (TESTS=...), verbose, each test time-limited.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-t}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 ${LIMIT:-1100} python -u -m pytest ${TESTS:-tests} -v -s -m gpu --timeout 1100 --timeout-method thread ${PYARGS:-} > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest.log | tail -40
exit $rc
