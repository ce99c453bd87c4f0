# Round 4: fused plane-march matrix powers (k_powers_planes).  Parity tests,
# then the headline and the 5-pt leg with the fused powers on / off and the
# planes per block.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r04_powers}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    -k "fused_planes or matrix_powers or spmv" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
b() {  # name env... : one short bench, summary line
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --no-legs --steps 20 $BARGS > $O/b_$tag.json 2> $O/b_$tag.err
  local rc=$?
  python - $O/b_$tag.json $tag <<'PY'
import json,sys
d=json.load(open(sys.argv[1]))
print(sys.argv[2], round(d['value'],1), 'spmv_avg_us', round(d['spmv_avg_us'],1), 'lpp', d.get('spmv_launches_per_step'),
      'GB/s', round(d['spmv_gbps']), {k: round(v,3) for k,v in d['kernel_ms_per_step'].items()},
      'diag', round(d['diagnostics_on']['outer_iters_per_s'],1))
PY
  return $rc
}
BARGS="--workload lap3d_215"
b l3_def || exit 1
BARGS="--workload lap2d_3162"
for Z in 8 16 32; do b l2_f2_z$Z CAL_POW_FMAX=2 CAL_POW_Z=$Z || exit 1; done
for Z in 16 32; do b l2_f3_z$Z CAL_POW_FMAX=3 CAL_POW_Z=$Z || exit 1; done
b l2_f1 CAL_POW_FMAX=1 || exit 1
exit 0

b l3_f1 CAL_POW_FMAX=1 || exit 1
for Z in 8 16 24; do b l3_z$Z CAL_POW_Z=$Z || exit 1; done
BARGS="--workload lap2d_3162"
b l2_f1 CAL_POW_FMAX=1 || exit 1
for Z in 8 12 16 24; do b l2_z$Z CAL_POW_Z=$Z || exit 1; done
b l2_f2 CAL_POW_FMAX=2 CAL_POW_Z=16 || exit 1
