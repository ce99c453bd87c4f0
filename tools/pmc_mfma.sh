cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/mfma
export TMPDIR=/tmp
cd /tmp
timeout -k 10 60 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/mfma/counters.txt 2>&1
grep -i "mfma\|GRBM_GUI_ACTIVE\|SQ_BUSY_CYCLES\|FLOPS\|VALU_MFMA" $GRAFT_REPO_ROOT/gpurun_out/mfma/counters.txt | head -40 > $GRAFT_REPO_ROOT/gpurun_out/mfma/mfma_names.txt
timeout -k 10 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/mfma/pass1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/mfma/pass1.log 2>&1
echo rc=$?
