# fused-TSQR parity tests, then a same-box A/B of the TSQR leg over env
# settings (SETS: ';'-separated env assignments, "-" = defaults), twice each
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-fold_ab}
mkdir -p $O
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_tsqr.py tests/test_gpu_parity.py tests/test_gpu_config4.py} -x -v -m gpu -k "${KSEL:-tsqr or project_and_normalize or backends or config4}" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed|Error" $O/pytest.log | tail -5
if [ $rc -ne 0 ]; then exit $rc; fi
IFS=';' read -ra S <<< "${SETS:--;CAL_FOLD_SIDE=0 CAL_FOLD_ROOT=0}"
for rep in 1 2; do
  i=0
  for set in "${S[@]}"; do
    i=$((i+1))
    [ "$set" = "-" ] && set=""
    env $set timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_${i}_$rep.json 2> $O/bench_${i}_$rep.err || exit $?
    python3 -c "
import json;d=json.load(open('$O/bench_${i}_$rep.json'));t=d.get('tsqr_step',{})
print('[$set]', 'rep $rep', 'bench', round(d['value'],1), 'tsqr', round(t.get('outer_iters_per_s',0),1), 'diag', round(d['diagnostics_on']['outer_iters_per_s'],1))"
  done
done
