#!/bin/bash
# round 6: same-box A/B of the IRL's normest on its own stream (test build:
# CAL_TEST_NORMEST_SYNC=1 runs the synchronous normest_dev)
set -o pipefail
O=gpurun_out/r06/${TAG:-irl_ab}
mkdir -p $O
for rep in 1 2 3; do
for v in async sync; do
  if [ $v = sync ]; then E="CAL_TEST_NORMEST_SYNC=1"; else E=""; fi
  env CAL_LIBRARY=testhooks $E timeout -k 10 300 python bench.py --driver irl --workload circuit_1259 --no-cpu-baseline --steps 5 --warmup 1 > $O/irl_$v.$rep.json 2> $O/irl_$v.$rep.err || exit $?
  python3 -c "
import json; i=json.load(open('$O/irl_$v.$rep.json'))
print('%-5s %.2f solves/s %.2f ms restarts %d norm %r' % ('$v', i['value'], i['ms_per_step'], i['num_restarts'], i['top_eigs'][:2]))"
done
done
