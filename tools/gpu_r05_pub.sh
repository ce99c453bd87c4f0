# Round 5: single-rank reductions published to host-mapped memory with the projection
# coefficients (k_reduce_pub) -- parity subset, IRL A/B (CAL_REDUCE_PUB_OFF=1 is the old path).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r05_pub}
mkdir -p $O
K="prologue or project or restart or normalize or orth or irl or parity or distributed or exhausted or selective"
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "$K" > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for v in on off host; do
    unset CAL_REDUCE_PUB_OFF CAL_REDUCE_PUB_HOST; [ $v = off ] && export CAL_REDUCE_PUB_OFF=1; [ $v = host ] && export CAL_REDUCE_PUB_HOST=1
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-legs --steps 5 --workload circuit_1259 --driver irl > $O/irl_$v.$rep.json 2> $O/irl_$v.$rep.err || exit $?
    python3 -c "
import json; d=json.load(open('$O/irl_$v.$rep.json'))
print('%-4s' % '$v', round(d['value'],2), {k: round(x) for k, x in d['roofline']['gbps_by_class'].items()}, round(d['time_split']['untimed_share'],3), {k: round(x, 2) for k, x in d['kernel_ms_per_solve'].items()})"
  done
done
