#!/bin/bash
# round 6: k_passb_wide probe builds (variant_pbw1: loads + LDS rows, no MFMA;
# variant_pbw2: loads only) against the library, kernel durations on the
# 'full' leg (timing only: the probe builds' Grams are wrong)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06/${TAG:-pbw_probe}
mkdir -p $O
for v in base pbw1 pbw2; do
  if [ $v = base ]; then L=""; else L="variant_$v"; fi
  CAL_LIBRARY=$L LEG_ORTH=full LEG_STEPS=14 LEG_WARMUP=1 LEG_REPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 tools/leg_only.py > $O/$v.json 2> $O/$v.err || exit $?
  echo "== $v"; python3 tools/kstats.py $O/$v/run_kernel_stats.csv 12 | grep passb_wide
done
