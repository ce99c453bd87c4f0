#!/bin/bash
# RCCL multi-rank: config 5's topology (irregular CSR, compact ghosts) on the one-GPU box
mkdir -p gpurun_out/rccl
timeout -k 10 500 python -u -m pytest tests/test_gpu_rccl_multirank.py -x -v -s --timeout 200 --timeout-method thread \
  -k "case3 or case4 or case5" 2>&1 | tee gpurun_out/rccl/pytest_circ.log
