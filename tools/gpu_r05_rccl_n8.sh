#!/bin/bash
# the driver's SCALE command at N = 8 (bench.py --gpus 8, default workload), all 8 ranks on the
# one GPU over RCCL's socket transport (CAL_RCCL_HOSTID_PER_RANK=1): a rehearsal, not a scaling number
mkdir -p gpurun_out/rccl
( while true; do sleep 30; date >> gpurun_out/rccl/heartbeat_n8.txt; done ) &
HB=$!
T0=$(date +%s)
CAL_RCCL_HOSTID_PER_RANK=1 timeout -k 10 600 python -u bench.py --gpus ${NG:-8} \
  > gpurun_out/rccl/bench_n${NG:-8}.json 2> gpurun_out/rccl/bench_n${NG:-8}.err
rc=$?
kill $HB
echo "rc=$rc wall=$(( $(date +%s) - T0 )) s"
tail -c 1500 gpurun_out/rccl/bench_n${NG:-8}.json
grep -v "amdgpu.ids\|socket.cpp\|Gloo\|RCCL version\|HIP version\|ROCm version\|Hostname\|Librccl" gpurun_out/rccl/bench_n${NG:-8}.err | tail -30
exit $rc
