# Round 5: the staged apply (+ next-block Gram) -- parity subsets on the production build and
# the staged-apply variant, then IRL A/B: base (fused step on / off), variant as1 (plain applies staged).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r05_stage}
mkdir -p $O
K="project or restart or normalize or orth or irl or parity"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "$K" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
CAL_LIBRARY=variant_as1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "$K" > $O/tests_as1.log 2>&1
rc=$?; tail -2 $O/tests_as1.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in on off as1 as1off; do
    unset CAL_APPLY_GRAM_OFF CAL_LIBRARY
    case $v in off) export CAL_APPLY_GRAM_OFF=1;; as1) export CAL_LIBRARY=variant_as1;; as1off) export CAL_LIBRARY=variant_as1 CAL_APPLY_GRAM_OFF=1;; esac
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-legs --steps 5 --workload circuit_1259 --driver irl > $O/irl_$v.$rep.json 2> $O/irl_$v.$rep.err || exit $?
    python3 -c "
import json; d=json.load(open('$O/irl_$v.$rep.json'))
print('%-7s' % '$v', round(d['value'],2), {k: round(x) for k, x in d['roofline']['gbps_by_class'].items()}, round(d['time_split']['untimed_share'],3), {k: round(x, 2) for k, x in d['kernel_ms_per_solve'].items()})"
  done
done
