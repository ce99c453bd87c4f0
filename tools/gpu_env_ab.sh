# Same-box A/B of one environment switch (VAR, values VALS, default
# CAL_LANE_SLOTS 0/1, interleaved twice): the diagnostics-only run under
# rocprofv3 kernel stats (tools/diag_only.py) and the bench's JSON line
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-env_ab}
VAR=${VAR:-CAL_LANE_SLOTS}
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  for v in ${VALS:-0 1}; do
    env $VAR=$v DIAG_REPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${v}_$rep -o run -- \
        python3 tools/diag_only.py > $O/diag_${v}_$rep.json 2> $O/diag_${v}_$rep.err || exit $?
    env $VAR=$v timeout -k 10 300 python bench.py --no-cpu-baseline ${BARGS:-} > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || exit $?
    echo "$VAR=$v rep=$rep diag $(cat $O/diag_${v}_$rep.json | head -c 300)"
    python3 -c "
import json;d=json.load(open('$O/bench_${v}_$rep.json'))
print(' bench', round(d['value'],1), 'spmv_b2b', d['spmv_kernel_back_to_back']['avg_us'], 'spmv_avg', round(d['spmv_avg_us'],2), 'diag', round(d['diagnostics_on']['outer_iters_per_s'],1), 'tsqr', round(d.get('tsqr_step',{}).get('outer_iters_per_s',0),1))"
  done
done
