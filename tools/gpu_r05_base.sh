# Round 5 baseline on this round's box: the default line (no CPU baseline) and the
# diagnostics-only rocprof (residual / Ritz apply kernel times).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r05_base}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit $?
python3 -c "import json;d=json.load(open('$O/bench.json'));print('line', round(d['value'],1), 'tsqr', round(d['tsqr_step']['outer_iters_per_s'],1), 'diag', round(d['diagnostics_on']['outer_iters_per_s'],1), 'csr', round(d['csr_step']['outer_iters_per_s'],1), 'irl', round(d['irl']['solves_per_s'],2))"
cd /tmp && DIAG_REPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/diag_only.py > $O/prof.log 2>&1
echo "prof rc=$?"
