# Round 4: plane-march SpMV + residual (prefetched keys, uniform slot values): parity tests first,
# then diagnostics timing, and the default bench with the plane SpMV off / Z = 8, 16, 32.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r04_planes2}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -v -m gpu --timeout 600 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
DIAG_REPS=2 timeout -k 10 300 python tools/diag_only.py > $O/diag.json 2> $O/diag.err || exit $?
echo "diag $(cat $O/diag.json)"
for Z in 0 8 16 32; do
  CAL_SPMV_PLANES=$Z timeout -k 10 300 python bench.py --no-cpu-baseline --no-legs > $O/bench_z$Z.json 2> $O/bench_z$Z.err || exit $?
  python3 -c "import json;d=json.load(open('$O/bench_z$Z.json'));print('Z=$Z', round(d['value'],1), 'spmv us', round(d['spmv_avg_us'],1), 'b2b', round(d.get('spmv_kernel_back_to_back',{}).get('avg_us',0),1), 'diag', round(d['diagnostics_on']['outer_iters_per_s'],1))"
done
cd /tmp && DIAG_REPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/diag_only.py > $O/prof.log 2>&1
echo "prof rc=$?"
