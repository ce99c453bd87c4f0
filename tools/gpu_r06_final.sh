# Round 6 verification: (PART=tests) the full GPU suite and smoke(); (PART=bench) the default
# bench line and a rocprofv3 kernel-trace/stats run of the headline (no legs, no CPU baseline).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r06_bench}
mkdir -p $O
export TMPDIR=/tmp
if [ "$PART" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
  rc=$?; tail -2 $O/smoke.log; exit $rc
fi
timeout -k 10 700 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
python3 - <<PY
import json
d=json.load(open('$O/bench.json'))
print('line', round(d['value'],1), 'roof', round(d['roofline']['frac'],3))
for k in ('tsqr_step','csr_step','lap2d_3162_step','lap2d_1000_step','full_step'):
    L=d.get(k,{}); print(k, round(L.get('outer_iters_per_s',0),1), 'share', L.get('kernel_share'), 'gbps', {a:round(b or 0) for a,b in L.get('kernel_gbps',{}).items()}, L.get('roofline',{}).get('kernel_class'))
print('irl', round(d['irl']['solves_per_s'],2), d['irl']['roofline']['kernel_class'], round(d['irl']['roofline']['achieved']), d['irl']['time_split'])
print('diag', round(d['diagnostics_on']['outer_iters_per_s'],1), 'cpu', d['cpu_baseline']['value'], d['cpu_baseline'].get('min'), d['cpu_baseline'].get('max'))
PY
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-legs > $O/bench_prof.json 2> $O/bench_prof.err
echo "prof rc=$?"
