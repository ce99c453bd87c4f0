# Round 4: size-based non-temporal Q stores in pass B and k_fold_down.
# Block-orthogonalisation parity tests, then the default line twice.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r04_nt2}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    tests/test_gpu_tsqr.py tests/test_gpu_fullsize.py -k "project or tsqr or lanczos or fullsize" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 400 python bench.py --no-cpu-baseline > $O/b_$i.json 2> $O/b_$i.err || exit 1
  python - $O/b_$i.json <<'PY'
import json,sys
d=json.load(open(sys.argv[1]))
print(round(d['value'],1), 'frac', round(d['roofline']['frac'],3), 'tsqr', round(d['tsqr_step']['outer_iters_per_s'],1), 'csr', round(d['csr_step']['outer_iters_per_s'],1),
      'lap2d', round(d['lap2d_3162_step']['outer_iters_per_s'],1), 'irl', round(d['irl']['solves_per_s'],2), 'diag', round(d['diagnostics_on']['outer_iters_per_s'],1),
      {k: round(v,3) for k,v in d['tsqr_step']['kernel_ms_per_step'].items()})
PY
done
