# Round 4 A/B: pass B's Q stores non-temporal (CAL_PASSB_NT=1) vs plain, alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r04_passb_nt}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fullsize.py \
    -k "csr_nontemporal or fullsize_vs_omp" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do for v in 0 1; do
  CAL_PASSB_NT=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-legs --steps 30 > $O/b_${v}_$i.json 2> $O/b_${v}_$i.err || exit 1
  python - $O/b_${v}_$i.json $v <<'PY'
import json,sys
d=json.load(open(sys.argv[1]))
print('NT', sys.argv[2], round(d['value'],1), {k: round(v,3) for k,v in d['kernel_ms_per_step'].items()}, 'spmv_us', round(d['spmv_avg_us'],1), 'gram_us', round(d['roofline']['avg_launch_us'],1))
PY
done; done
