# rocprofv3 kernel trace (per-launch timestamps) of one bench configuration:
#   BARGS="--normalize tsqr" TAG=trace_tsqr bash tools/gpu_trace.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-trace}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-legs --steps ${STEPS:-10} --warmup 2 ${BARGS:-} > $O/bench.json 2> $O/bench.err
rc=$?
echo rc=$rc
cut -c1-200 $O/bench.json
exit $rc
