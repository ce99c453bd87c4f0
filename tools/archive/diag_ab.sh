# A/B of the deferred Ritz diagnostics: bench.py --no-legs (diagnostics_on
# leg included) under each CAL_RESID_CPB, plus one rocprofv3 kernel-stats run.
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-diag_ab}
mkdir -p $O
export TMPDIR=/tmp
for cpb in ${CPBS:-2 4 8}; do
    CAL_RESID_CPB=$cpb timeout -k 10 200 python bench.py --no-cpu-baseline --no-legs > $O/bench_cpb$cpb.json 2> $O/bench_cpb$cpb.err || exit $?
    python -c "import json,sys; d=json.load(open('$O/bench_cpb$cpb.json')); print('cpb', $cpb, d['value'], d['diagnostics_on']['outer_iters_per_s'])"
done
cd /tmp && CAL_RESID_CPB=${PROF_CPB:-4} timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-legs > $O/prof.log 2>&1 || exit $?
python3 $GRAFT_REPO_ROOT/tools/kstats.py $O/prof/run_kernel_stats.csv 12
