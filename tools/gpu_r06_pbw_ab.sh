#!/bin/bash
# round 6: the fused pass B + wide Gram, production vs a kernels.hip variant (VARIANTS), full leg
set -o pipefail
O=gpurun_out/r06/${TAG:-pbw_ab}
mkdir -p $O
for rep in 1 2; do
for v in ${VARIANTS:-base pf}; do
  if [ "$v" = base ]; then L=""; else L="variant_$v"; fi
  CAL_LIBRARY=$L LEG_ORTH=full LEG_STEPS=14 LEG_REPS=1 timeout -k 10 300 python tools/leg_only.py > $O/full_$v.$rep.json 2> $O/full_$v.$rep.err || exit $?
  python3 -c "
import json; f=json.load(open('$O/full_$v.$rep.json'))[0]
print('%-5s full %.1f it/s gram %.3f apply %.3f' % ('$v', f['outer_iters_per_s'], f['kernel_ms_per_step']['gram'], f['kernel_ms_per_step']['apply']))"
done
done
