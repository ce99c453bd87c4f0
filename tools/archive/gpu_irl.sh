# IRL parity tests, bench line and kernel profile (BASELINE config 5 stand-in)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/irl
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests -q -m gpu -k "impl_restarted" > gpurun_out/irl/pt.log 2>&1 && \
timeout -k 10 400 python bench.py --workload circuit_1259 --driver irl > gpurun_out/irl/bench.json 2> gpurun_out/irl/bench.err && \
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/irl/prof -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --workload circuit_1259 --driver irl --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/irl/prof.log 2>&1
echo rc=$?
