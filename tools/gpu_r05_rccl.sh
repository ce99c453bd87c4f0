#!/bin/bash
# RCCL with several ranks on the one-GPU box (NCCL_HOSTID per rank, sockets over loopback)
mkdir -p gpurun_out/rccl
timeout -k 10 600 python -u -m pytest tests/test_gpu_rccl_multirank.py -x -v -s --timeout 300 --timeout-method thread \
  > gpurun_out/rccl/pytest.log 2>&1
rc=$?
tail -40 gpurun_out/rccl/pytest.log
exit $rc
