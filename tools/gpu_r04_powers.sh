# Round 4: fused plane-march matrix powers (k_powers_planes).  Parity tests,
# then the headline and the 5-pt leg with the fused powers on / off.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r04_powers}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    -k "fused_planes or matrix_powers or spmv" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
for W in lap3d_215 lap2d_3162; do
  for F in 1 4; do
    CAL_POW_FMAX=$F timeout -k 10 300 python bench.py --no-cpu-baseline --no-legs --workload $W --steps 20 \
        > $O/bench_${W}_f$F.json 2> $O/bench_${W}_f$F.err
    rc=$?; echo "bench $W F=$F rc=$rc"; cut -c1-260 $O/bench_${W}_f$F.json
    [ $rc -eq 0 ] || exit $rc
  done
done
for Z in 8 27 48; do
  CAL_POW_Z=$Z timeout -k 10 300 python bench.py --no-cpu-baseline --no-legs --workload lap3d_215 --steps 20 \
      > $O/bench_lap3d_z$Z.json 2> $O/bench_lap3d_z$Z.err
  echo "bench lap3d Z=$Z rc=$?"; cut -c1-200 $O/bench_lap3d_z$Z.json
done
CAL_SPMV_CSR=hoist timeout -k 10 200 python tools/csr_variant.py > $O/csr_hoist.json 2>&1
echo "csr rc=$?"; cat $O/csr_hoist.json
