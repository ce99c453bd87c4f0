# Round 5: Gram shapes of the IRL driver, then A/B of the row-staged Gram variants.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r05_gram2}
mkdir -p $O
CAL_LOG_GRAM_SHAPES=1 timeout -k 10 300 python bench.py --workload circuit_1259 --driver irl --no-cpu-baseline --steps 1 --warmup 0 > $O/shapes.json 2> $O/shapes.err || exit $?
grep "^gram " $O/shapes.err | sort | uniq -c | sort -rn > $O/shapes.txt; head -30 $O/shapes.txt
TAG=${TAG:-r05_gram2}/ab REPS=${REPS:-2} STEPS=${STEPS:-5} BENCH_ARGS="--workload circuit_1259 --driver irl" VARIANTS="${VARIANTS:-base g0 g4 g4b}" bash tools/ab_variants.sh
