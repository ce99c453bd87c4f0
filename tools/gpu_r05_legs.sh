# Round 5: kernel traces of single bench legs (tools/leg_only.py) for gap analysis.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r05_legs}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for spec in ${SPECS:-csr:local:auto:lap3d_215}; do
  IFS=: read F OR NZ WLD <<< "$spec"
  LEG_FORMAT=$F LEG_ORTH=$OR LEG_NORMALIZE=$NZ LEG_WORKLOAD=$WLD timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$F.$OR.$NZ.$WLD -o run -- python3 $GRAFT_REPO_ROOT/tools/leg_only.py > $O/$F.$OR.$NZ.$WLD.log 2>&1 || exit $?
  echo "== $spec"; grep outer_iters $O/$F.$OR.$NZ.$WLD.log | tail -1
  python3 $GRAFT_REPO_ROOT/tools/trace_gaps.py $O/$F.$OR.$NZ.$WLD/run_kernel_trace.csv 3 || true
done
