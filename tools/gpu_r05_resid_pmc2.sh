# Round 5: the final plane-march residual (k_resid_planes v4) alone: kernel trace, then PMC
# passes (FETCH_SIZE; TA/TD busy; LDS, waits and VALU), one rocprofv3 --pmc run per group.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r05_resid_pmc2}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
R="--kernel-include-regex k_resid_planes"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $GRAFT_REPO_ROOT/tools/resid_only.py > $O/trace.log 2>&1 || exit $?
grep plane_info $O/trace.log
timeout -s KILL 120 rocprofv3 $R --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 $GRAFT_REPO_ROOT/tools/resid_only.py > $O/fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 $R --pmc TA_BUSY_avr TA_TA_BUSY_sum TD_BUSY_avr TD_TD_BUSY_sum GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/tatd -o run -- python3 $GRAFT_REPO_ROOT/tools/resid_only.py > $O/tatd.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 $R --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/sq -o run -- python3 $GRAFT_REPO_ROOT/tools/resid_only.py > $O/sq.log 2>&1 || exit $?
echo done
