# Round 5: MFMA counters of the Gram sweeps (P1, pass A) and the Ritz apply on the current
# kernels (bench.py, lap3d_215, diagnostics leg included), one --pmc pass, kernels filtered.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r05_pmc_mfma}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 300 rocprofv3 --kernel-include-regex "k_rowapply|k_apply_mt" --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/pass1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-legs > $O/pass1.log 2>&1
echo "pmc rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-legs > $O/trace.log 2>&1
echo "trace rc=$?"
