# bench line (with the CPU baseline) + a kernel-stats profile of the
# diagnostics-on run alone (tools/diag_only.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-dp}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --no-legs > $O/bench.json 2> $O/bench.err && \
timeout -k 10 200 python tools/diag_only.py > $O/diag.json 2> $O/diag.err && \
cd /tmp && DIAG_REPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python3 $GRAFT_REPO_ROOT/tools/diag_only.py > $O/prof.log 2>&1
echo rc=$?
