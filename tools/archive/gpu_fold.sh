# fused-TSQR checks: TSQR / projectAndNormalize / multirank parity tests, then
# the bench's TSQR leg under rocprofv3 kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-fold}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_tsqr.py tests/test_gpu_parity.py} -x -v -m gpu -k "${KSEL:-tsqr or project_and_normalize or backends}" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed|Error" $O/pytest.log | tail -30
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline ${BARGS:-} > $O/bench.json 2> $O/bench.err && \
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline ${BARGS:-} > $O/prof.log 2>&1
rc=$?
echo rc=$rc
python3 -c "
import json;d=json.load(open('$O/bench.json'));t=d.get('tsqr_step',{})
print(d['value'], json.dumps(t)[:900])"
exit $rc
