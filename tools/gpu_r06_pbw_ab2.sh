#!/bin/bash
# round 6: the bench's full_step configuration (W = 1, K = 14: k = 2..15) on one box:
# production, test build fused, test build separate (CAL_TEST_PASSB_WIDE_OFF)
set -o pipefail
O=gpurun_out/r06/${TAG:-pbw_ab2}
mkdir -p $O
for rep in 1 2 3; do
for v in prod fused sep; do
  case $v in prod) E="";; fused) E="CAL_LIBRARY=testhooks";; sep) E="CAL_LIBRARY=testhooks CAL_TEST_PASSB_WIDE_OFF=1";; esac
  env $E LEG_ORTH=full LEG_STEPS=14 LEG_WARMUP=1 LEG_REPS=1 timeout -k 10 300 python tools/leg_only.py > $O/full_$v.$rep.json 2> $O/full_$v.$rep.err || exit $?
  python3 -c "
import json; f=json.load(open('$O/full_$v.$rep.json'))[0]
print('%-5s full %.1f it/s %.3f ms kernels %s' % ('$v', f['outer_iters_per_s'], f['ms_per_step'], {k: round(x,3) for k,x in f['kernel_ms_per_step'].items()}))"
done
done
