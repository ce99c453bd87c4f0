#!/bin/bash
# round 6: normest chunks as replayed graphs against direct launches
# (CAL_TEST_NEST_DIRECT, test build) and the production library, on the
# config-5 IRL bench, alternating, one box
set -o pipefail
O=gpurun_out/r06/${TAG:-nest_ab}
mkdir -p $O
for rep in 1 2 3; do
for v in prod graph direct; do
  case $v in prod) E="";; graph) E="CAL_LIBRARY=testhooks";; direct) E="CAL_LIBRARY=testhooks CAL_TEST_NEST_DIRECT=1";; esac
  env $E timeout -k 10 300 python bench.py --driver irl --workload circuit_1259 --no-cpu-baseline --steps 3 --warmup 1 > $O/irl_$v.$rep.json 2> $O/irl_$v.$rep.err || exit $?
  python3 -c "
import json; i=json.load(open('$O/irl_$v.$rep.json'))
print('%-6s irl %.2f solves/s split %s restarts %d' % ('$v', i['value'], {k: round(x, 3) for k, x in i['time_split'].items()}, i['num_restarts']))"
done
done
