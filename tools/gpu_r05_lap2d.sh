# Round 5: the full GPU suite, then a kernel trace of the lap2d_1000 leg (config 2) for its
# launch-boundary share.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r05_lap2d}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
cd /tmp
LEG_WORKLOAD=lap2d_1000 LEG_STEPS=100 LEG_REPS=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $GRAFT_REPO_ROOT/tools/leg_only.py > $O/leg.json 2> $O/leg.err
echo "trace rc=$?"
cat $O/leg.json
