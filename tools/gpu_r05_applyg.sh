#!/bin/bash
# A/B: columns in flight per thread in the wide row apply (k_apply_rows, CAL_APPLY_ROWS_G 8 / 16 / 32)
# on the 'full' leg of lap3d_215 and on the IRL
set -o pipefail
O=gpurun_out/applyg; mkdir -p $O
for rep in 1 2; do for v in base g16 g32; do
  if [ $v = base ]; then L=""; else L="variant_$v"; fi
  CAL_LIBRARY=$L LEG_ORTH=full LEG_STEPS=14 LEG_REPS=1 timeout -k 10 300 python tools/leg_only.py > $O/full_${v}_$rep.json 2>$O/full_${v}_$rep.err || { tail -5 $O/full_${v}_$rep.err; exit 1; }
  echo "full $v $rep $(python3 -c "import json; d=json.load(open('$O/full_${v}_$rep.json'))[-1]; print(round(d['outer_iters_per_s'],1), {k: round(x,3) for k,x in d['kernel_ms_per_step'].items()})")"
done; done
for v in base g16 g32; do
  if [ $v = base ]; then L=""; else L="variant_$v"; fi
  CAL_LIBRARY=$L timeout -k 10 200 python bench.py --workload circuit_1259 --driver irl --no-cpu-baseline --steps 5 > $O/irl_$v.json 2>$O/irl_$v.err || exit 1
  echo "irl $v $(python3 -c "import json; d=json.load(open('$O/irl_$v.json')); print(round(d['value'],2), d['kernel_ms_per_solve'])")"
done
