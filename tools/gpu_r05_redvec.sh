#!/bin/bash
# A/B: the reduce-then-update vector kernels (normest's k_nrm_div, the prologue's k_pro_div) on 1024
# blocks (library) against 4096 (variant_rv4096); the IRL solve rate and its top eigenvalues
set -o pipefail
O=gpurun_out/redvec; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "fused_bitexact" > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2 3; do for v in base rv4096; do
  if [ $v = base ]; then L=""; else L="variant_$v"; fi
  CAL_LIBRARY=$L timeout -k 10 200 python bench.py --workload circuit_1259 --driver irl --no-cpu-baseline --steps 5 > $O/irl_${v}_$rep.json 2>$O/irl_${v}_$rep.err || exit 1
  echo "$v $rep $(python3 -c "import json; d=json.load(open('$O/irl_${v}_$rep.json')); print(round(d['value'],2), d['top_eigs'], d['num_restarts'])")"
done; done
