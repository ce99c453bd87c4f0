# FETCH_SIZE of the batched residual kernel at several block shapes
# (CAL_RESID_CPB x CAL_RESID_PPT), one --pmc pass each
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/rfetch
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for cfg in "1 4" "1 1" "2 1"; do
    set -- $cfg
    CAL_RESID_CPB=$1 CAL_RESID_PPT=$2 DIAG_REPS=0 timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv \
        -d $O/f_$1_$2 -o run -- python3 $GRAFT_REPO_ROOT/tools/diag_only.py > $O/f_$1_$2.log 2>&1 || exit 1
done
echo rc=$?
