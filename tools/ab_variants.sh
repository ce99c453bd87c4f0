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
ks = d.get('kernel_ms_per_step') or d.get('kernel_ms_per_solve') or {}
ex = ''
if 'spmv_avg_us' in d:
    ex = 'spmv %.1f b2b %.1f diag %.1f' % (d['spmv_avg_us'], d['spmv_kernel_back_to_back']['avg_us'], d['diagnostics_on']['outer_iters_per_s'])
elif 'roofline' in d:
    ex = 'gbps %s split %s' % ({k: round(x) for k, x in d['roofline'].get('gbps_by_class', {}).items()}, d.get('time_split'))
print('%-8s'%'$v', round(d['value'],2), ex, {k: round(x*1e3,1) for k,x in ks.items()})"
done
done
