#!/bin/bash
# config 4 at full size over RCCL (2 ranks on the one-GPU box)
mkdir -p gpurun_out/rccl
timeout -k 10 700 python -u -m pytest tests/test_gpu_rccl_multirank.py -x -v -s --timeout 600 --timeout-method thread \
  -k "config4" 2>&1 | tee gpurun_out/rccl/pytest_cfg4.log
