# Round 5: k_resid_planes alone (tools/resid_only.py): kernel trace, then PMC passes
# (instruction mix, waits, LDS, fetch), one rocprofv3 --pmc run per group.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r05_resid_pmc}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
R="--kernel-include-regex k_resid_planes"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $GRAFT_REPO_ROOT/tools/resid_only.py > $O/trace.log 2>&1 || exit $?
grep plane_info $O/trace.log
timeout -s KILL 120 rocprofv3 $R --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --output-format csv -d $O/p1 -o run -- python3 $GRAFT_REPO_ROOT/tools/resid_only.py > $O/p1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 $R --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE --output-format csv -d $O/p2 -o run -- python3 $GRAFT_REPO_ROOT/tools/resid_only.py > $O/p2.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 $R --pmc FETCH_SIZE --output-format csv -d $O/p3 -o run -- python3 $GRAFT_REPO_ROOT/tools/resid_only.py > $O/p3.log 2>&1 || exit $?
echo done
