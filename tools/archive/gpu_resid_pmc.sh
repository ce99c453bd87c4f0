# PMC passes on the batched Ritz-residual kernel and the pair SpMV
# (diagnostics-only run, tools/diag_only.py): SQ issue/wait split, then
# texture-path busy counters.  One pass per counter group, each under its own
# time limit.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-resid_pmc}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
cd /tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_INSTS_SALU"
P2="${P2:-TA_BUSY_avr TA_TA_BUSY_sum TD_BUSY_avr TD_TD_BUSY_sum GRBM_GUI_ACTIVE GRBM_COUNT}"
P3="${P3:-TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum}"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  DIAG_REPS=0 timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex "resid_multi|k_spmv_pair<1" --output-format csv \
      -d $O/pmc$i -o run -- python3 $GRAFT_REPO_ROOT/tools/diag_only.py > $O/pmc$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
done
exit 0
