#!/bin/bash
# round 6: rocprof kernel stats of the 'full' leg (lap3d_215, 14 steps) and the IRL driver
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06/${TAG:-fullprof}
mkdir -p $O
LEG_ORTH=full LEG_STEPS=14 LEG_REPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/full -o run -- python3 tools/leg_only.py > $O/full.json 2> $O/full.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/irl -o run -- python3 bench.py --driver irl --workload circuit_1259 --no-cpu-baseline --steps 3 --warmup 1 > $O/irl.json 2> $O/irl.err || exit $?
find $O -name "*kernel_stats.csv" | head
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 python -u -m pytest tests/test_gpu_hooks.py::test_normest_and_irl_fused_bitexact "tests/test_gpu_parity.py" -k "impl_restarted or normest or periodic or full" -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -3 $O/pytest.log
