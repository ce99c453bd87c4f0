#!/bin/bash
# A/B of the two-chunks-in-flight Gram sweeps (CAL_ROWGRAM_PF2_MB=0 off, 192 on): config 2's leg,
# the bits of T, the IRL, then a kernel trace of the config-2 leg with PF2 (VGPRs, scratch)
set -o pipefail
O=gpurun_out/pf2; mkdir -p $O
for mb in 0 192; do CAL_ROWGRAM_PF2_MB=$mb timeout -k 10 120 python tools/pf2_check.py > $O/bits_$mb.txt 2>&1 || exit 1; done
cat $O/bits_*.txt
for rep in 1 2; do for mb in 0 192; do
  CAL_ROWGRAM_PF2_MB=$mb LEG_WORKLOAD=lap2d_1000 LEG_STEPS=100 LEG_REPS=2 timeout -k 10 200 python tools/leg_only.py > $O/cfg2_${mb}_$rep.json 2>$O/cfg2_${mb}_$rep.err || exit 1
  echo "cfg2 pf2mb=$mb rep=$rep $(python3 -c "import json; print([round(x['outer_iters_per_s'],1) for x in json.load(open('$O/cfg2_${mb}_$rep.json'))], json.load(open('$O/cfg2_${mb}_$rep.json'))[-1]['kernel_ms_per_step'])")"
done; done
for mb in 0 192; do
  CAL_ROWGRAM_PF2_MB=$mb timeout -k 10 200 python bench.py --workload circuit_1259 --driver irl --no-cpu-baseline --steps 5 > $O/irl_$mb.json 2>$O/irl_$mb.err || exit 1
  echo "irl pf2mb=$mb $(python3 -c "import json; d=json.load(open('$O/irl_$mb.json')); print(round(d['value'],2), d['kernel_ms_per_solve'])")"
done
cd /tmp && export TMPDIR=/tmp
CAL_ROWGRAM_PF2_MB=192 LEG_WORKLOAD=lap2d_1000 LEG_STEPS=100 LEG_REPS=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/leg_only.py > $GRAFT_REPO_ROOT/$O/prof.json 2>$GRAFT_REPO_ROOT/$O/prof.err
echo "prof rc=$?"
