#!/bin/bash
# the 2-rank RCCL line with its multi-rank IRL leg, output streamed to files
mkdir -p gpurun_out/rccl
( while true; do sleep 30; date >> gpurun_out/rccl/heartbeat.txt; done ) &
HB=$!
CAL_BENCH_STAGE_LIMIT=${LIM:-240} CAL_RCCL_HOSTID_PER_RANK=1 timeout -k 10 400 python -u bench.py --gpus 2 --steps 3 --warmup 1 --workload lap3d_40 \
  > gpurun_out/rccl/bench_lap3d_40_irl.json 2> gpurun_out/rccl/bench_lap3d_40_irl.err
rc=$?
kill $HB
echo "rc=$rc"
tail -c 2500 gpurun_out/rccl/bench_lap3d_40_irl.json
grep -v "amdgpu.ids\|socket.cpp\|Gloo" gpurun_out/rccl/bench_lap3d_40_irl.err | grep -B2 -A40 "exceeded" | head -120
exit $rc
