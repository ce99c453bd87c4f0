# Round 4: the plane-march residual (k_resid_planes): full GPU suite, diagnostics-only timing,
# rocprof kernel stats of the diagnostics run, then the default bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r04_planes}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu --timeout 600 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
DIAG_REPS=2 timeout -k 10 300 python tools/diag_only.py > $O/diag.json 2> $O/diag.err || exit $?
echo "diag $(cat $O/diag.json)"
cd /tmp && DIAG_REPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/diag_only.py > $O/prof.log 2>&1
echo "prof rc=$?"
cd $GRAFT_REPO_ROOT && timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-200 $O/bench.json
exit $rc
