# Round verification: gpu tests, smoke, default bench (with CPU baseline), rocprofv3 kernel stats.
# Each GPU step is time-limited and the chain stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-round}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err && \
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $O/prof.log 2>&1
rc=$?
echo rc=$rc
tail -3 $O/pytest.log; cat $O/smoke.log | tail -1; cut -c1-300 $O/bench.json
exit $rc
