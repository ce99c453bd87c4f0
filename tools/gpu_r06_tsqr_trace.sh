#!/bin/bash
# round 6: kernel trace of the TSQR leg (config 3 as named, lap3d_215)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06/${TAG:-tsqr_trace}
mkdir -p $O
LEG_NORMALIZE=tsqr LEG_STEPS=10 LEG_REPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- python3 tools/leg_only.py > $O/leg.json 2> $O/leg.err || exit $?
cat $O/leg.json
