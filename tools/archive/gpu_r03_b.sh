# new parity tests + multirank + roctx marker trace of a short bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-b}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py -v -s -m gpu -k "harness or complex_pair or multirank" --timeout 600 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed|error in" $O/pytest.log | tail -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv -d $O/mark -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-legs --steps 5 --warmup 1 > $O/mark.json 2> $O/mark.err
echo "mark rc=$?"; ls $O/mark
