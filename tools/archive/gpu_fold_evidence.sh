# fused-TSQR evidence: kernel stats of the bench (TSQR leg included), then
# FETCH_SIZE and WRITE_SIZE of the up / down sweeps (one PMC pass each)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-fold_ev}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit $?
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C --kernel-include-regex "k_fold_(up|down)\(" --output-format csv -d $O/pmc_$C -o run -- \
      python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 5 --warmup 1 > $O/pmc_$C.log 2>&1
  rc=$?; echo "$C rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
done
