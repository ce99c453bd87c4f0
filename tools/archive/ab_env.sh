# A/B a tuning environment variable over the default bench (no CPU baseline):
#   VAR=CAL_SPMV_NT_TAIL VALS="0 2 4" REPS=2 bash tools/ab_env.sh
cd $GRAFT_REPO_ROOT
O=gpurun_out/ab_${VAR}
mkdir -p $O
for rep in $(seq 1 ${REPS:-2}); do for v in $VALS; do
env $VAR=$v timeout -k 10 200 python bench.py --no-cpu-baseline --steps ${STEPS:-30} ${BARGS:-} > $O/v${v}_r${rep}.json 2> $O/err.txt || exit 1
python -c "import json;d=json.load(open('$O/v${v}_r${rep}.json'));print('$VAR=$v rep $rep', round(d['value'],1), {k: round(x, 4) for k, x in d['kernel_ms_per_step'].items()})"
done; done
