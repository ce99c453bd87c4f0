#!/bin/bash
# round 6: the wide-read probe on the BW = 8 staging, then the 'full' leg and
# the IRL driver on the production build
set -o pipefail
O=gpurun_out/r06/${TAG:-gram2}
mkdir -p $O
timeout -k 10 240 ./tools/wide_read_probe > $O/wide_read_probe.json 2>&1 || exit $?
cut -c1-60,300- $O/wide_read_probe.json | sed 's/"rows.*panel16/ .. "panel16/'
for rep in 1 2; do
    LEG_ORTH=full LEG_STEPS=14 LEG_REPS=1 timeout -k 10 300 python tools/leg_only.py > $O/full.$rep.json 2> $O/full.$rep.err || exit $?
    timeout -k 10 300 python bench.py --driver irl --workload circuit_1259 --no-cpu-baseline --steps 3 --warmup 1 > $O/irl.$rep.json 2> $O/irl.$rep.err || exit $?
    python3 -c "
import json; f=json.load(open('$O/full.$rep.json'))[0]; i=json.load(open('$O/irl.$rep.json'))
print('full %.1f it/s gram %.3f apply %.3f | irl %.2f solves/s gram %.0f GB/s split %.3f' % (f['outer_iters_per_s'], f['kernel_ms_per_step']['gram'], f['kernel_ms_per_step']['apply'], i['value'], i['roofline']['gbps_by_class']['gram'], i['time_split']['untimed_share']))"
done
