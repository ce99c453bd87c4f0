# Round 5: row-staged narrow Gram (k_gram_rows) -- parity subset, then A/B on the IRL driver.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r05_gram}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "${KSEL:-gram or project or restart or normalize or orth}" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
TAG=${TAG:-r05_gram}/ab REPS=${REPS:-2} STEPS=${STEPS:-5} BENCH_ARGS="--workload circuit_1259 --driver irl" VARIANTS="${VARIANTS:-base g0 g8 gb2}" bash tools/ab_variants.sh
