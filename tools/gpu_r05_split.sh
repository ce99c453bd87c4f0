#!/bin/bash
# A/B: 65..128-column Grams split over two row-staged launches (library) against k_gram_lds
# (variant_nosplit) on the 'full' leg of lap3d_215, then the 'full'-mode parity tests
set -o pipefail
O=gpurun_out/split; mkdir -p $O
for rep in 1 2; do for v in base nosplit; do
  if [ $v = base ]; then L=""; else L="variant_$v"; fi
  CAL_LIBRARY=$L LEG_ORTH=full LEG_STEPS=14 LEG_REPS=1 timeout -k 10 300 python tools/leg_only.py > $O/full_${v}_$rep.json 2>$O/full_${v}_$rep.err || { tail -5 $O/full_${v}_$rep.err; exit 1; }
  echo "$v $rep $(python3 -c "import json; d=json.load(open('$O/full_${v}_$rep.json'))[-1]; print(round(d['outer_iters_per_s'],1), {k: round(x,3) for k,x in d['kernel_ms_per_step'].items()})")"
done; done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_distributed.py -x -q --timeout 300 --timeout-method thread -k "full or periodic or selective or gram or restart" > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; exit $rc
