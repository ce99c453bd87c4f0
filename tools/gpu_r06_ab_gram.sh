#!/bin/bash
# round 6: A/B of the k_gram_rows register-slot depth (CAL_GRAM_ROWS_NSLOT)
# on the 'full' leg (lap3d_215) and the IRL driver (circuit_1259)
set -o pipefail
O=gpurun_out/r06/${TAG:-ab_gram}
mkdir -p $O
for rep in 1 2; do
for v in ${VARIANTS:-base ns3 ns4}; do
    if [ "$v" = base ]; then L=""; else L="variant_$v"; fi
    CAL_LIBRARY=$L LEG_ORTH=full LEG_STEPS=14 LEG_REPS=1 timeout -k 10 300 python tools/leg_only.py > $O/full_$v.$rep.json 2> $O/full_$v.$rep.err || exit $?
    CAL_LIBRARY=$L timeout -k 10 300 python bench.py --driver irl --workload circuit_1259 --no-cpu-baseline --steps 3 --warmup 1 > $O/irl_$v.$rep.json 2> $O/irl_$v.$rep.err || exit $?
    python3 -c "
import json; f=json.load(open('$O/full_$v.$rep.json'))[0]; i=json.load(open('$O/irl_$v.$rep.json'))
print('%-5s full %.1f it/s gram %.3f apply %.3f | irl %.2f solves/s gram %.0f GB/s split %.3f' % ('$v', f['outer_iters_per_s'], f['kernel_ms_per_step']['gram'], f['kernel_ms_per_step']['apply'], i['value'], i['roofline']['gbps_by_class']['gram'], i['time_split']['untimed_share']))"
done
done
