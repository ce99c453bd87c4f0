# parity tests of the block orthogonalisation + a kernel-stats profile of bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/qp
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -k "${TESTK:-orth or normalize or project or ca_lanczos}" > $O/pt.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err && \
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 10 > $O/prof.log 2>&1
echo rc=$?
