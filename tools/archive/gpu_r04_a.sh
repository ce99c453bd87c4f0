# Round 4, call A: the new full-size parity tests (config 3 with TSQR, lap2d_3162) and the default bench
# line with its new legs (lap2d_3162_step, irl). Each GPU step time-limited; stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r04a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -x -v -s -m gpu --timeout 600 --timeout-method thread > $O/pytest_fullsize.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $O/pytest_fullsize.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-400 $O/bench.json
[ $rc -eq 0 ] || exit $rc
