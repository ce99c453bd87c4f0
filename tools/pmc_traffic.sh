# HBM traffic counters for the hot kernels, one rocprofv3 --pmc pass per
# counter group (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE cannot share
# a pass; no trace domains alongside --pmc).  Run on the GPU box:
#   bash tools/pmc_traffic.sh            -> gpurun_out/pmc/<tag>_<group>/...
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
STEPS=${STEPS:-3}
run() {  # tag group counters... -- cmd
    local tag=$1 grp=$2; shift 2
    local ctr=()
    while [ "$1" != "--" ]; do ctr+=("$1"); shift; done
    shift
    timeout -k 10 300 rocprofv3 --pmc "${ctr[@]}" --output-format csv -d $OUT/${tag}_${grp} -o run -- "$@" \
        > $OUT/${tag}_${grp}.log 2>&1
    local rc=$?
    echo "$tag $grp rc=$rc"
    return $rc
}
for grp in fetch write hit; do
    case $grp in
        fetch) C=(FETCH_SIZE) ;;
        write) C=(WRITE_SIZE) ;;
        hit) C=(TCC_HIT_sum TCC_MISS_sum) ;;
    esac
    if [ -z "$BENCH_ONLY" ]; then
        run spmv $grp "${C[@]}" -- python3 $GRAFT_REPO_ROOT/tools/spmv_sweep.py --reps 10 || exit $?
    fi
    run bench $grp "${C[@]}" -- python3 $GRAFT_REPO_ROOT/bench.py --steps $STEPS --warmup 1 --no-cpu-baseline $BENCH_ARGS || exit $?
done
cd $GRAFT_REPO_ROOT && python3 tools/traffic_json.py gpurun_out/pmc --out gpurun_out/pmc/spmv_traffic.json > /dev/null
