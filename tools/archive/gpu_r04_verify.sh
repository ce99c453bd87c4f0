# Round 4 verification: full GPU suite, smoke, default bench (with CPU baseline), rocprof kernel
# stats of the headline.  Each GPU step time-limited; stops at the first hard failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r04_verify}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu --timeout 600 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-200 $O/bench.json
[ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $O/prof.log 2>&1
echo "prof rc=$?"
