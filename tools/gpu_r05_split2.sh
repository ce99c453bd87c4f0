#!/bin/bash
# A/B: 65..128-column Grams in 64-column (library) against 32-column launches
# (variant_s2) on the 'full' leg of lap3d_215, then the 'full'-mode parity tests
set -o pipefail
O=gpurun_out/split2; mkdir -p $O
for rep in 1 2; do for v in base s2; do
  if [ $v = base ]; then L=""; else L="variant_$v"; fi
  CAL_LIBRARY=$L LEG_ORTH=full LEG_STEPS=14 LEG_REPS=1 timeout -k 10 300 python tools/leg_only.py > $O/full_${v}_$rep.json 2>$O/full_${v}_$rep.err || { tail -5 $O/full_${v}_$rep.err; exit 1; }
  echo "$v $rep $(python3 -c "import json; d=json.load(open('$O/full_${v}_$rep.json'))[-1]; print(round(d['outer_iters_per_s'],1), {k: round(x,3) for k,x in d['kernel_ms_per_step'].items()})")"
done; done
