# Round 4 quick A/B: the plane-march residual and SpMV kernel times (rocprof of the diagnostics-only
# run) and the default bench line with the plane SpMV off (Z=0) and on (Z=16).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r04_quick}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "spmv or powers or lanczos_ex or fullsize" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && DIAG_REPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/diag_only.py > $O/prof.log 2>&1
echo "prof rc=$?"
cd $GRAFT_REPO_ROOT
for Z in ${ZS:-0 16}; do
  CAL_SPMV_PLANES=$Z timeout -k 10 300 python bench.py --no-cpu-baseline --no-legs > $O/bench_z$Z.json 2> $O/bench_z$Z.err || exit $?
  python3 -c "import json;d=json.load(open('$O/bench_z$Z.json'));print('Z=$Z', round(d['value'],1), 'spmv us', round(d['spmv_avg_us'],1), 'b2b', round(d.get('spmv_kernel_back_to_back',{}).get('avg_us',0),1), 'diag', round(d['diagnostics_on']['outer_iters_per_s'],1))"
done
