# Round 5: lap2d_1000 (n = 1e6, a multiple of 64) with two rows of ld slack (plane march) vs none.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r05_ld}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "planes or config2 or fullsize or lap2d" > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in slack noslack; do
    unset CAL_LD_NOSLACK; [ $v = noslack ] && export CAL_LD_NOSLACK=1
    LEG_WORKLOAD=lap2d_1000 LEG_STEPS=100 LEG_REPS=2 timeout -k 10 300 python tools/leg_only.py > $O/$v.$rep.json 2> $O/$v.$rep.err || exit $?
    echo "$v $(python3 -c "import json; print([(round(x['outer_iters_per_s']), {k: round(v*1e3,1) for k, v in x['kernel_ms_per_step'].items()}) for x in json.load(open('$O/$v.$rep.json'))])")"
  done
done
