# Round 5: HBM counter traffic (FETCH_SIZE x2, WRITE_SIZE, separate passes) of the IRL's kernels
# (circuit_1259, one solve after a warm-up) -- the row-staged Gram, the staged apply and its fused
# variants against their algorithmic bytes.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r05_pmc_irl}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
R="--kernel-include-regex k_gram_rows|k_apply_stage|k_apply_rows|k_spmv<|k_rowapply"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload circuit_1259 --driver irl --no-cpu-baseline --steps 1 --warmup 1 > $O/trace.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 $R --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload circuit_1259 --driver irl --no-cpu-baseline --steps 1 --warmup 1 > $O/fetch.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 $R --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload circuit_1259 --driver irl --no-cpu-baseline --steps 1 --warmup 1 > $O/write.log 2>&1 || exit $?
echo done
