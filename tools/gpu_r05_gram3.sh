# Round 5: full GPU suite with the row-staged Gram, then A/B against the k_gram build (g0)
# on the headline line and the IRL driver.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r05_gram3}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
TAG=${TAG:-r05_gram3}/irl REPS=2 STEPS=5 BENCH_ARGS="--workload circuit_1259 --driver irl" VARIANTS="base g0" bash tools/ab_variants.sh || exit $?
TAG=${TAG:-r05_gram3}/head REPS=2 VARIANTS="base g0" bash tools/ab_variants.sh
