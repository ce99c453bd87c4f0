#!/bin/bash
# kernel trace + stats of the IRL driver alone (config 5)
mkdir -p gpurun_out/irl_prof
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/irl_prof -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --workload circuit_1259 --driver irl --no-cpu-baseline --steps 3 --warmup 1 \
  > $GRAFT_REPO_ROOT/gpurun_out/irl_prof/bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/irl_prof/bench.err
echo "rc=$?"
