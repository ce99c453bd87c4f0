# diagnostics-on A/B of the batched residual kernel's shape
# (CAL_RESID_CPB Ritz pairs per block x CAL_RESID_PPT row pairs per thread)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-rab}
mkdir -p $O
for cfg in "4 4" "1 1" "1 4" "2 1" "2 2" "4 1" "4 2" "8 1" "4 4"; do
    set -- $cfg
    CAL_RESID_CPB=$1 CAL_RESID_PPT=$2 timeout -k 10 200 python tools/diag_only.py > $O/d_$1_$2.json 2> $O/d_$1_$2.err || exit 1
    echo cpb $1 ppt $2 $(cat $O/d_$1_$2.json)
done
