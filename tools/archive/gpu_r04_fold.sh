# Round 4: the compact-WY fused TSQR (tsqr_fold.hip).  Kernel probe, the fold's parity tests,
# config 3 at full size, the TSQR-normalize bench with its rocprof kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r04_fold}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 ./tools/fold_probe_dw3 > $O/probe.txt 2>&1
rc=$?; echo "probe rc=$rc"; cat $O/probe.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_tsqr.py \
    tests/test_gpu_parity.py -k "tsqr or project or lanczos" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 280 --timeout-method thread tests/test_gpu_fullsize.py \
    -k config3 > $O/pytest_c3.log 2>&1
rc=$?; echo "pytest c3 rc=$rc"; tail -3 $O/pytest_c3.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-legs --normalize tsqr > $O/bench_tsqr.json 2> $O/prof.log
echo "prof rc=$?"; cut -c1-300 $O/bench_tsqr.json
cd $GRAFT_REPO_ROOT
if [ -n "$WITH_C5" ]; then
  # progress marks for the long multi-rank case (its ranks print at the end)
  ( for i in $(seq 14); do sleep 60; date >> $O/heartbeat_c5; done ) &
  HB=$!
  timeout -k 10 800 python -u -m pytest -x -v -s --timeout 780 --timeout-method thread tests/test_gpu_multirank.py \
      -k config5 > $O/pytest_c5.log 2>&1
  rc=$?; kill $HB 2>/dev/null; echo "pytest c5 rc=$rc"; tail -3 $O/pytest_c5.log
fi
