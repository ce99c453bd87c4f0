# Round 5: fused norms-before Gram -- parity subset, IRL line + trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r05_gram4}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "${KSEL:-project or restart or normalize or orth or irl or parity}" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
TAG=${TAG:-r05_gram4}/irl REPS=2 STEPS=5 BENCH_ARGS="--workload circuit_1259 --driver irl" VARIANTS="base" bash tools/ab_variants.sh || exit $?
TAG=${TAG:-r05_gram4}/trace bash tools/gpu_r05_irl.sh
