# HBM fetch counters and L2 hit rate of the diagnostics-on kernels
# (tools/diag_only.py), one --pmc pass per counter group
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_diag
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
DIAG_REPS=0 timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- \
    python3 $GRAFT_REPO_ROOT/tools/diag_only.py > $OUT/fetch.log 2>&1 && \
DIAG_REPS=0 timeout -k 10 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/hit -o run -- \
    python3 $GRAFT_REPO_ROOT/tools/diag_only.py > $OUT/hit.log 2>&1
echo rc=$?
