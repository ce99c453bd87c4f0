# Round 5: the bench tests (contract, two ranks, watchdog) and the full default line.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r05_bench}
mkdir -p $O
export TMPDIR=/tmp
if [ -z "$NOTEST" ]; then
timeout -k 10 900 python -u -m pytest tests/test_gpu_bench.py -x -v -m gpu --timeout 400 --timeout-method thread > $O/pytest_bench.log 2>&1
rc=$?; echo "pytest bench rc=$rc"; tail -3 $O/pytest_bench.log
[ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
python3 - <<PY
import json
d=json.load(open('$O/bench.json'))
print('line', round(d['value'],1), 'roof', round(d['roofline']['frac'],3))
for k in ('tsqr_step','csr_step','lap2d_3162_step','lap2d_1000_step','full_step'):
    L=d.get(k,{}); print(k, round(L.get('outer_iters_per_s',0),1), 'share', round(L.get('kernel_share',0),3), 'gbps', {a:round(b or 0) for a,b in L.get('kernel_gbps',{}).items()}, L.get('roofline',{}).get('kernel_class'))
print('irl', round(d['irl']['solves_per_s'],2), d['irl']['roofline']['kernel_class'], round(d['irl']['roofline']['achieved']), d['irl']['time_split'])
print('diag', round(d['diagnostics_on']['outer_iters_per_s'],1), 'cpu', d['cpu_baseline']['value'], d['cpu_baseline']['min'], d['cpu_baseline']['max'])
PY
