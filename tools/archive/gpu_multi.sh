# Several measurements in one call: gpu tests (restart/IRL/diagnostics parity),
# diagnostics A/B, 'full' orth rate, the IRL bench.  Each step time-limited;
# the chain stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-multi}
mkdir -p $O
export TMPDIR=/tmp
if [ "$PTK" != "none" ]; then
    timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread -k "${PTK:-lanczos or restart or irl}" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
    tail -2 $O/pytest.log
fi
for cpb in ${CPBS-4}; do
    CAL_RESID_CPB=$cpb timeout -k 10 200 python bench.py --no-cpu-baseline --no-legs > $O/bench_cpb$cpb.json 2> $O/bench_cpb$cpb.err || exit 1
    python -c "import json; d=json.load(open('$O/bench_cpb$cpb.json')); print('cpb', $cpb, round(d['value'],1), round(d['diagnostics_on']['outer_iters_per_s'],1))"
done
for o in ${ORTHS-full}; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-legs --orth $o > $O/orth_$o.json 2> $O/orth_$o.err || exit 1
    python -c "import json;d=json.load(open('$O/orth_$o.json'));print('$o', round(d['value'],1), d['kernel_ms_per_step'])"
done
if [ -n "$IRL" ]; then
    timeout -k 10 400 python bench.py --workload circuit_1259 --driver irl --no-cpu-baseline > $O/irl.json 2> $O/irl.err || exit 1
    python -c "import json;d=json.load(open('$O/irl.json'));print('irl', d['value'], d['unit'])"
fi
if [ -n "$PROF" ]; then
    cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
        python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-legs $PROF_ARGS > $O/prof.log 2>&1 || exit 1
    python3 $GRAFT_REPO_ROOT/tools/kstats.py $O/prof/run_kernel_stats.csv 14
fi
