# Round 5: fused block-MGS step (k_apply_gram) -- parity subset, then IRL with it on / off.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r05_ag}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "${KSEL:-project or restart or normalize or orth or irl or parity}" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in on off; do
    if [ $v = off ]; then export CAL_APPLY_GRAM_OFF=1; else unset CAL_APPLY_GRAM_OFF; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-legs --steps 5 --workload circuit_1259 --driver irl > $O/$v.$rep.json 2> $O/$v.$rep.err || exit $?
    python3 -c "
import json; d=json.load(open('$O/$v.$rep.json'))
print('$v', round(d['value'],2), {k: round(x) for k, x in d['roofline']['gbps_by_class'].items()}, d['time_split'], d['kernel_ms_per_solve'])"
  done
done
