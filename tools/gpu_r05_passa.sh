# Round 5: pass A of the no-Qp CholQR2 normalize on the staged kernel (k_apply_stage<..., 3>) -- parity
# subset, IRL A/B (CAL_PASSA_STAGE_OFF=1 keeps k_rowapply).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r05_passa}
mkdir -p $O
K="headline or harness or exhausted or prologue or project or restart or normalize or orth or irl or parity or distributed or exhausted or selective"
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "$K" > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for v in on off; do
    unset CAL_PASSA_STAGE_OFF; [ $v = off ] && export CAL_PASSA_STAGE_OFF=1
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-legs --steps 5 --workload circuit_1259 --driver irl > $O/irl_$v.$rep.json 2> $O/irl_$v.$rep.err || exit $?
    python3 -c "
import json; d=json.load(open('$O/irl_$v.$rep.json'))
print('%-4s' % '$v', round(d['value'],2), {k: round(x) for k, x in d['roofline']['gbps_by_class'].items()}, round(d['time_split']['untimed_share'],3), {k: round(x, 2) for k, x in d['kernel_ms_per_solve'].items()})"
  done
done
