# A/B on one box: bench.py (no CPU baseline) under each setting of an env knob
#   KNOB=CAL_EXP VALUES="0 1" bash tools/ab_bench.sh
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2; do
for v in $VALUES; do
    env $KNOB=$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/ab_$v.log 2>&1 || exit 1
    python3 -c "
import json; d=json.loads(open('gpurun_out/ab_$v.log').read().strip().splitlines()[-1])
print('$KNOB=$v', round(d['value'],1), {k: round(x*1e3,1) for k,x in d['kernel_ms_per_step'].items()})"
done
done
