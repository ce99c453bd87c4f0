# A/B of the batched residual kernel: CAL_RESID_PPT x CAL_RESID_CPB, diagnostics-on rate
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-diag_ab2}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread -k "lanczos and (diag or parity or config4)" > $O/pt.log 2>&1 || { tail -20 $O/pt.log; exit 1; }
tail -1 $O/pt.log
for cfg in ${CFGS:-"1 4" "4 4" "8 4" "4 8" "8 8"}; do
    set -- $cfg
    CAL_RESID_PPT=$1 CAL_RESID_CPB=$2 timeout -k 10 200 python bench.py --no-cpu-baseline --no-legs > $O/b_$1_$2.json 2> $O/b_$1_$2.err || exit 1
    python -c "import json; d=json.load(open('$O/b_$1_$2.json')); print('ppt', $1, 'cpb', $2, round(d['value'],1), round(d['diagnostics_on']['outer_iters_per_s'],1))"
done
