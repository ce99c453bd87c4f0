# A/B of kernel-tuning builds on one box: bench.py (no CPU baseline, no legs) with
# CAL_LIBRARY=variant_X for each X in VARIANTS ("base" = the production library),
# REPS rounds in alternating order.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-ab_variants}
mkdir -p $O
for rep in $(seq 1 ${REPS:-2}); do
for v in $VARIANTS; do
    if [ "$v" = base ]; then L=""; else L="variant_$v"; fi
    CAL_LIBRARY=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-legs --steps ${STEPS:-20} $BENCH_ARGS > $O/$v.$rep.json 2> $O/$v.$rep.err || exit $?
    python3 -c "
import json; d=json.load(open('$O/$v.$rep.json'))
print('%-8s'%'$v', round(d['value'],1), 'spmv', round(d['spmv_avg_us'],1), 'b2b', round(d['spmv_kernel_back_to_back']['avg_us'],1), 'diag', round(d['diagnostics_on']['outer_iters_per_s'],1), {k: round(x*1e3,1) for k,x in d['kernel_ms_per_step'].items()})"
done
done
