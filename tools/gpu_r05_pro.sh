# Round 5: fused prologue recurrence (k_axpy_dot) -- parity subset, IRL A/B (fused / separate,
# production / staged-apply variant).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r05_pro}
mkdir -p $O
K="prologue or project or restart or normalize or orth or irl or parity or distributed"
[ -n "$SKIP_TESTS" ] || timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "$K" > $O/tests.log 2>&1
rc=$?; [ -n "$SKIP_TESTS" ] || tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in on off as0; do
    unset CAL_PROLOGUE_FUSED CAL_LIBRARY
    case $v in off) export CAL_PROLOGUE_FUSED=0;; as0) export CAL_LIBRARY=variant_as0;; esac
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-legs --steps 5 --workload circuit_1259 --driver irl > $O/irl_$v.$rep.json 2> $O/irl_$v.$rep.err || exit $?
    python3 -c "
import json; d=json.load(open('$O/irl_$v.$rep.json'))
print('%-7s' % '$v', round(d['value'],2), {k: round(x) for k, x in d['roofline']['gbps_by_class'].items()}, round(d['time_split']['untimed_share'],3), {k: round(x, 2) for k, x in d['kernel_ms_per_solve'].items()})"
  done
done
