# A/B of the batched Ritz-residual kernel: the 2-D grid (CAL_RESID_PERS=0)
# against the persistent XCD-ranged kernel at 1 / 2 / 4 pairs per pass,
# diagnostics-on runs only (tools/diag_only.py, lap3d_215, t = 15)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-resid_ab2}
mkdir -p $O
export TMPDIR=/tmp
for v in "0 2" "1 1" "1 2" "1 4"; do
  set -- $v
  CAL_RESID_PERS=$1 CAL_RESID_PCPB=$2 DIAG_REPS=2 timeout -k 10 300 python tools/diag_only.py > $O/diag_p$1_c$2.json 2> $O/diag_p$1_c$2.err || exit $?
  echo "pers=$1 pcpb=$2 $(cat $O/diag_p$1_c$2.json)"
done
