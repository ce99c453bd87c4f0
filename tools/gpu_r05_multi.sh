# Round 5: fused block-MGS step (k_apply_gram) and adaptive planes per block -- parity
# subsets, IRL with the fusion on / off, the lap2d_1000 leg, the CSR floor probe.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r05_multi}
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "${KSEL:-project or restart or normalize or orth or irl or parity or planes or config2}" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in on off; do
    if [ $v = off ]; then export CAL_APPLY_GRAM_OFF=1; else unset CAL_APPLY_GRAM_OFF; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-legs --steps 5 --workload circuit_1259 --driver irl > $O/irl_$v.$rep.json 2> $O/irl_$v.$rep.err || exit $?
    python3 -c "
import json; d=json.load(open('$O/irl_$v.$rep.json'))
print('$v', round(d['value'],2), {k: round(x) for k, x in d['roofline']['gbps_by_class'].items()}, d['time_split'], d['kernel_ms_per_solve'])"
  done
done
unset CAL_APPLY_GRAM_OFF
LEG_WORKLOAD=lap2d_1000 LEG_STEPS=100 LEG_REPS=3 timeout -k 10 300 python tools/leg_only.py > $O/lap2d_1000_leg.json 2> $O/lap2d_1000_leg.err || exit $?
cat $O/lap2d_1000_leg.json
timeout -k 10 120 ./tools/csr_floor_probe > $O/csr_floor_probe.json || exit $?
cat $O/csr_floor_probe.json
