#!/bin/bash
mkdir -p gpurun_out/rccl
for W in 2 4 8; do
  timeout -k 10 260 python -u tools/rccl_irl_ranks.py $W > gpurun_out/rccl/irl_ranks_$W.txt 2>&1 || { echo "W=$W failed"; grep -v "amdgpu.ids\|socket.cpp\|Gloo" gpurun_out/rccl/irl_ranks_$W.txt | tail -40; exit 1; }
  grep -v "amdgpu.ids\|socket.cpp\|Gloo\|RCCL version\|HIP version\|ROCm version\|Hostname\|Librccl" gpurun_out/rccl/irl_ranks_$W.txt
done
