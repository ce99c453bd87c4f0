# Bench lines + rocprofv3 kernel stats (csv) for the headline and the IRL.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/ev
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > $O/head.json 2> $O/head.err && \
timeout -k 10 300 python bench.py --workload lap2d_3162 --no-cpu-baseline > $O/lap2d.json 2> $O/lap2d.err && \
timeout -k 10 300 python bench.py --workload circuit_1259 --no-cpu-baseline > $O/circ.json 2> $O/circ.err && \
timeout -k 10 400 python bench.py --workload circuit_1259 --driver irl > $O/irl.json 2> $O/irl.err && \
cd /tmp && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_head -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $O/prof_head.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_irl -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --workload circuit_1259 --driver irl --no-cpu-baseline > $O/prof_irl.log 2>&1
echo rc=$?
