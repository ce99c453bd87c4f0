# Round 5: plane march v4 (E/O split LDS windows, own pair in registers, host wave masks,
# NEG1 stencils, unrolled by 3): plane tests, residual-only trace, diagnostics trace, line.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r05_planes2}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_planes.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_planes.log 2>&1
rc=$?; echo "pytest planes rc=$rc"; tail -3 $O/pytest_planes.log
[ $rc -eq 0 ] || exit $rc
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rtrace -o run -- python3 $GRAFT_REPO_ROOT/tools/resid_only.py > $O/rtrace.log 2>&1 || exit $?
grep plane_info $O/rtrace.log
DIAG_REPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/diag_only.py > $O/prof.log 2>&1
echo "prof rc=$?"; grep outer_iters $O/prof.log | tail -1
cd $GRAFT_REPO_ROOT
if [ -n "$PARITY" ]; then
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q -m gpu -k "spmv or powers or lanczos or fullsize" --timeout 600 --timeout-method thread > $O/pytest_par.log 2>&1
rc=$?; echo "pytest parity rc=$rc"; tail -2 $O/pytest_par.log
[ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit $?
python3 -c "import json;d=json.load(open('$O/bench.json'));print('line', round(d['value'],1), 'tsqr', round(d['tsqr_step']['outer_iters_per_s'],1), 'diag', round(d['diagnostics_on']['outer_iters_per_s'],1), 'csr', round(d['csr_step']['outer_iters_per_s'],1), 'irl', round(d['irl']['solves_per_s'],2), 'spmv_us', round(d['spmv_avg_us'],1), 'b2b', round(d['spmv_kernel_back_to_back']['avg_us'],1), 'lap2d', round(d['lap2d_3162_step']['outer_iters_per_s'],1))"
