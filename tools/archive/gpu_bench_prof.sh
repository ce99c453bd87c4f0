# bench (no CPU baseline) + rocprofv3 kernel trace of the same command, each step time-limited
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-bp}
mkdir -p $O
export TMPDIR=/tmp
${PRE:-true} && \
timeout -k 10 300 python bench.py --no-cpu-baseline ${BARGS:-} > $O/bench.json 2> $O/bench.err && \
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline ${BARGS:-} > $O/prof.log 2>&1
rc=$?
echo rc=$rc
cut -c1-260 $O/bench.json
exit $rc
