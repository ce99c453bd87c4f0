# Round 4: forced-decline / restart tests, then the residual kernel with and without the
# lane-shared +-1 slots (CAL_RESID_LANE): diagnostics-only rates, kernel stats, TA/TD PMC.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r04_resid2}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_tsqr.py tests/test_gpu_parity.py -x -v -s -m gpu -k "declined or restarted or backends" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "restarts:|passed|failed" $O/pytest.log | tail -4
[ $rc -eq 0 ] || exit $rc
for L in 0 1; do
  CAL_RESID_LANE=$L DIAG_REPS=2 timeout -k 10 300 python tools/diag_only.py > $O/diag_l$L.json 2> $O/diag_l$L.err || exit $?
  echo "lane=$L $(cat $O/diag_l$L.json)"
done
cd /tmp
for L in 0 1; do
  CAL_RESID_LANE=$L DIAG_REPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_l$L -o run -- python3 $GRAFT_REPO_ROOT/tools/diag_only.py > $O/prof_l$L.log 2>&1
  echo "prof lane=$L rc=$?"
  i=0
  for P in "TA_BUSY_avr TA_TA_BUSY_sum TD_BUSY_avr TD_TD_BUSY_sum GRBM_GUI_ACTIVE GRBM_COUNT" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_INSTS_SALU" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum"; do
    i=$((i+1))
    CAL_RESID_LANE=$L DIAG_REPS=0 timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex "k_resid_pairs" --output-format csv \
        -d $O/pmc_l${L}_$i -o run -- python3 $GRAFT_REPO_ROOT/tools/diag_only.py > $O/pmc_l${L}_$i.log 2>&1
    rc=$?
    echo "pmc lane=$L pass $i rc=$rc"
    if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
  done
done
exit 0
