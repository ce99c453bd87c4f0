#!/bin/bash
# round 6: a kernel + copy trace of the config-5 IRL bench (one timed solve) to
# place the untimed share (idle gaps between launches)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06/${TAG:-irl_trace}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/prof -o run -- python3 bench.py --driver irl --workload circuit_1259 --no-cpu-baseline --steps 1 --warmup 1 > $O/irl.json 2> $O/irl.err || exit $?
ls $O/prof
