# A/B of the diagnostics streams / chunks (CAL_DIAG_AUX, CAL_DIAG_CHUNKS)
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-diag_ab3}
mkdir -p $O
for cfg in "1 1" "1 2" "0 1" "0 2" "1 3"; do
    set -- $cfg
    CAL_DIAG_AUX=$1 CAL_DIAG_CHUNKS=$2 timeout -k 10 200 python bench.py --no-cpu-baseline --no-legs > $O/b_$1_$2.json 2> $O/b_$1_$2.err || exit 1
    python -c "import json; d=json.load(open('$O/b_$1_$2.json')); print('aux', $1, 'chunks', $2, round(d['value'],1), round(d['diagnostics_on']['outer_iters_per_s'],1))"
done
