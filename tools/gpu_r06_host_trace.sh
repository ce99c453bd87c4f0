#!/bin/bash
# round 6: kernel + HIP runtime API trace of the headline (no legs, no CPU
# baseline) to see whether a launch reaches the stream after its predecessor
# finished (host late) or before (device-side gap)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06/${TAG:-host_trace}
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline --no-legs --steps 20 > $O/bench.json 2> $O/bench.err || exit $?
ls $O/prof
