#!/bin/bash
# kernel trace of the TSQR-normalize leg alone (config 3 as named)
O=gpurun_out/tsqr_trace; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
LEG_NORMALIZE=tsqr LEG_STEPS=10 LEG_REPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O -o run -- python3 $GRAFT_REPO_ROOT/tools/leg_only.py > $GRAFT_REPO_ROOT/$O/leg.json 2>$GRAFT_REPO_ROOT/$O/leg.err
echo "rc=$?"; cat $GRAFT_REPO_ROOT/$O/leg.json
