# GPU check: gpu tests, smoke, bench, rocprofv3 kernel stats (each step time-limited)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
STEPS=${STEPS:-10}
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -6 gpurun_out/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps $STEPS --warmup 2 --no-cpu-baseline > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/bench.log | cut -c1-400
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps $STEPS --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1; echo "prof rc=$?"
