# Round 4: PMC passes on the library's plane-march residual (diagnostics-only run) and on the
# probe's k_res_zw (tools/resid_probe.hip), to compare what bounds each.  One pass per group.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r04_pmc_planes}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_LDS_DATA_FIFO_FULL GRBM_GUI_ACTIVE"
P3="TA_BUSY_avr TA_TA_BUSY_sum TD_BUSY_avr TD_TD_BUSY_sum GRBM_GUI_ACTIVE GRBM_COUNT"
P4="FETCH_SIZE GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  DIAG_REPS=0 timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex "k_resid_planes" --output-format csv \
      -d $O/lib$i -o run -- python3 $GRAFT_REPO_ROOT/tools/diag_only.py > $O/lib$i.log 2>&1
  rc=$?; echo "lib pass $i rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex "k_res_zw" --output-format csv \
      -d $O/probe$i -o run -- $GRAFT_REPO_ROOT/tools/resid_probe 32 > $O/probe$i.log 2>&1
  rc=$?; echo "probe pass $i rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
exit 0
