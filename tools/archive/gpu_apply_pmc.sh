# PMC passes on the Ritz-vector apply (k_apply_mt) in the diagnostics-only
# run: issue / wait split and MFMA busy, then LDS and VMEM activity
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-apply_pmc}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU_MFMA_F64 GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_DATA_FIFO_FULL SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  DIAG_REPS=0 timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex "apply_mt" --output-format csv \
      -d $O/pmc$i -o run -- python3 $GRAFT_REPO_ROOT/tools/diag_only.py > $O/pmc$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
