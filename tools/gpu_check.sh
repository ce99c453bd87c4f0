cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest.log
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 400 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench.log 2>&1; rc2=$?; echo "bench rc=$rc2"; tail -3 gpurun_out/bench.log
  if [ $rc2 -eq 0 ]; then
    cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1; echo "prof rc=$?"
    find $GRAFT_REPO_ROOT/gpurun_out/prof -name "*stats*" | head
  fi
fi
