#!/bin/bash
# round 6: kernel traces of the full leg (W = 1, K = 14) with the fused pass B
# (test build) and with the separate sweeps (CAL_TEST_PASSB_WIDE_OFF)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06/${TAG:-pbw_trace}
mkdir -p $O
for v in fused sep; do
  if [ $v = sep ]; then export CAL_TEST_PASSB_WIDE_OFF=1; fi
  CAL_LIBRARY=testhooks LEG_ORTH=full LEG_STEPS=14 LEG_WARMUP=1 LEG_REPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/$v -o run -- python3 tools/leg_only.py > $O/$v.json 2> $O/$v.err || exit $?
done
