# Round 4 timing experiment: plane-march kernels with (CAL_PLANES_NOMASK=0) and without (=1, wrong
# results) the boundary-row selects, and the plane SpMV at Z = 8 / 16 / 32.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r04_nomask}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for M in 0 1; do
  CAL_PLANES_NOMASK=$M DIAG_REPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof$M -o run -- python3 $GRAFT_REPO_ROOT/tools/diag_only.py > $O/prof$M.log 2>&1
  echo "nomask=$M rc=$?"
done
cd $GRAFT_REPO_ROOT
for Z in 8 16 32; do
  CAL_SPMV_PLANES=$Z timeout -k 10 300 python bench.py --no-cpu-baseline --no-legs > $O/bench_z$Z.json 2> $O/bench_z$Z.err || exit $?
  python3 -c "import json;d=json.load(open('$O/bench_z$Z.json'));print('Z=$Z', round(d['value'],1), 'spmv us', round(d['spmv_avg_us'],1), 'b2b', round(d.get('spmv_kernel_back_to_back',{}).get('avg_us',0),1), 'diag', round(d['diagnostics_on']['outer_iters_per_s'],1))"
done
