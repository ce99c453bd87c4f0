#!/bin/bash
# A/B: the row Gram sweeps' grid (P1 / pass A, kRowGramBlocks 1024 library vs 512 variant_rg512) on
# config 2 (lap2d_1000), the IRL and the headline (no legs)
set -o pipefail
O=gpurun_out/rg; mkdir -p $O
for rep in 1 2; do for v in base rg512; do
  if [ $v = base ]; then L=""; else L="variant_$v"; fi
  CAL_LIBRARY=$L LEG_WORKLOAD=lap2d_1000 LEG_STEPS=100 LEG_REPS=2 timeout -k 10 200 python tools/leg_only.py > $O/cfg2_${v}_$rep.json 2>$O/cfg2_${v}_$rep.err || exit 1
  echo "cfg2 $v $rep $(python3 -c "import json; print([round(x['outer_iters_per_s'],1) for x in json.load(open('$O/cfg2_${v}_$rep.json'))])")"
  CAL_LIBRARY=$L timeout -k 10 200 python bench.py --workload circuit_1259 --driver irl --no-cpu-baseline --steps 5 > $O/irl_${v}_$rep.json 2>$O/irl_${v}_$rep.err || exit 1
  echo "irl $v $rep $(python3 -c "import json; d=json.load(open('$O/irl_${v}_$rep.json')); print(round(d['value'],2))")"
  CAL_LIBRARY=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-legs --steps 20 > $O/head_${v}_$rep.json 2>$O/head_${v}_$rep.err || exit 1
  echo "head $v $rep $(python3 -c "import json; d=json.load(open('$O/head_${v}_$rep.json')); print(round(d['value'],1))")"
done; done
