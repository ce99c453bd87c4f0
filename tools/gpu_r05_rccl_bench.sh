#!/bin/bash
# The driver's multi-rank bench line over RCCL, rehearsed on the one-GPU box
mkdir -p gpurun_out/rccl
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench.py -x -v -s --timeout 300 --timeout-method thread \
  -k "rccl_line" > gpurun_out/rccl/pytest_bench.log 2>&1 || { tail -30 gpurun_out/rccl/pytest_bench.log; exit 1; }
tail -5 gpurun_out/rccl/pytest_bench.log
CAL_RCCL_HOSTID_PER_RANK=1 timeout -k 10 700 python -u bench.py --gpus 2 --steps 10 --warmup 3 \
  > gpurun_out/rccl/bench_2rank_lap3d_215.json 2> gpurun_out/rccl/bench_2rank_lap3d_215.err
rc=$?
tail -c 3000 gpurun_out/rccl/bench_2rank_lap3d_215.json
exit $rc
