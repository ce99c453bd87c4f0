# fused-TSQR kernel probe: each FOLD_PROBE variant of k_fold_up timed at the bench shape
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-fprobe}
mkdir -p $O
for v in ${VARIANTS:-0_3 0_4 2_3 4_3 16_3}; do
  timeout -k 10 120 ./tools/fold_probe_$v >> $O/probe.txt 2>&1 || { echo "probe $v failed rc=$?"; cat $O/probe.txt; exit 1; }
done
cat $O/probe.txt
