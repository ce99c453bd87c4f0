# Round 5: headline / full-leg A/B of the staged plain apply (variant as1), IRL trace with it.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r05_stage2}
mkdir -p $O
TAG=${TAG:-r05_stage2}/head REPS=2 VARIANTS="base as1" bash tools/ab_variants.sh || exit $?
for v in base as1; do
  if [ $v = base ]; then L=""; else L="variant_$v"; fi
  CAL_LIBRARY=$L LEG_WORKLOAD=lap3d_215 LEG_ORTH=full LEG_STEPS=14 LEG_REPS=2 timeout -k 10 300 python tools/leg_only.py > $O/full_$v.json 2> $O/full_$v.err || exit $?
  echo "full $v $(python3 -c "import json; print([round(x['outer_iters_per_s'],1) for x in json.load(open('$O/full_$v.json'))])")"
done
export TMPDIR=/tmp
cd /tmp
CAL_LIBRARY=variant_as1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload circuit_1259 --driver irl --no-cpu-baseline > $O/irl.json 2> $O/irl.err
echo "irl rc=$?"
