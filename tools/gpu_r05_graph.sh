# Round 5: lap2d_1000 / lap3d_215 legs with the matrix powers as a HIP graph (CAL_POWERS_GRAPH=1) vs direct launches.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r05_graph}
mkdir -p $O
CAL_POWERS_GRAPH=1 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "config2 or planes or harness" > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in graph direct; do
    unset CAL_POWERS_GRAPH; [ $v = graph ] && export CAL_POWERS_GRAPH=1
    for w in lap2d_1000 lap3d_215; do
      LEG_WORKLOAD=$w LEG_STEPS=${STEPS:-100} LEG_REPS=2 timeout -k 10 300 python tools/leg_only.py > $O/$v.$w.$rep.json 2> $O/$v.$w.$rep.err || exit $?
      echo "$v $w $(python3 -c "import json; print([round(x['outer_iters_per_s']) for x in json.load(open('$O/$v.$w.$rep.json'))])")"
    done
  done
done
