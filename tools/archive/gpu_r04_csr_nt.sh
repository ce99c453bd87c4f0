# Round 4: CSR SpMV with non-temporal col/val loads when the matrix exceeds
# the Infinity Cache.  Parity tests of the SpMV and the restart drivers, the
# variant script, the default bench line (CSR leg, IRL leg).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r04_csr_nt}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    tests/test_gpu_fullsize.py -k "spmv or powers or restart or config5" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
CAL_SPMV_CSR=nt_auto timeout -k 10 200 python tools/csr_variant.py > $O/csr_nt_auto.json 2>&1
rc=$?; echo "csr rc=$rc"; cat $O/csr_nt_auto.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"
python - $O/bench.json <<'PY'
import json,sys
d=json.load(open(sys.argv[1]))
print('value', round(d['value'],1), 'tsqr', round(d['tsqr_step']['outer_iters_per_s'],1), 'csr', round(d['csr_step']['outer_iters_per_s'],1),
      'csr spmv us', round(d['csr_step']['spmv_avg_us'],1), 'irl', round(d['irl']['solves_per_s'],2),
      'lap2d', round(d['lap2d_3162_step']['outer_iters_per_s'],1), 'diag', round(d['diagnostics_on']['outer_iters_per_s'],1))
PY
