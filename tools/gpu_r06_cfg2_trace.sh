#!/bin/bash
# round 6: kernel trace of config 2 (lap2d_1000, s = 8 Newton, 'local')
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06/${TAG:-cfg2_trace}
mkdir -p $O
LEG_WORKLOAD=lap2d_1000 LEG_STEPS=100 LEG_REPS=1 timeout -k 10 300 python3 tools/leg_only.py > $O/leg_plain.json 2>&1 || exit $?
LEG_WORKLOAD=lap2d_1000 LEG_STEPS=100 LEG_REPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O -o run -- python3 tools/leg_only.py > $O/leg.json 2> $O/leg.err || exit $?
cat $O/leg_plain.json
