#!/bin/bash
# round 6: k_apply_rows tuning builds (VARIANTS, "base" = production) on the
# 'full' leg (W = 1, K = 14) and the IRL bench, alternating, one box
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06/${TAG:-apply_ab}
mkdir -p $O
for rep in 1 2; do
for v in $VARIANTS; do
  if [ "$v" = base ]; then L=""; else L="variant_$v"; fi
  CAL_LIBRARY=$L LEG_ORTH=full LEG_STEPS=14 LEG_WARMUP=1 LEG_REPS=1 timeout -k 10 300 python tools/leg_only.py > $O/full_$v.$rep.json 2> $O/full_$v.$rep.err || exit $?
  python3 -c "
import json; f=json.load(open('$O/full_$v.$rep.json'))[0]
print('%-8s full %.1f it/s %.3f ms kernels %s' % ('$v', f['outer_iters_per_s'], f['ms_per_step'], {k: round(x,3) for k,x in f['kernel_ms_per_step'].items()}))"
done
done
for rep in 1 2; do
for v in $VARIANTS; do
  if [ "$v" = base ]; then L=""; else L="variant_$v"; fi
  CAL_LIBRARY=$L timeout -k 10 300 python bench.py --driver irl --no-cpu-baseline --steps 5 > $O/irl_$v.$rep.json 2> $O/irl_$v.$rep.err || exit $?
  python3 -c "
import json; d=json.load(open('$O/irl_$v.$rep.json')); print('%-8s irl %.2f' % ('$v', d['value']))"
done
done
