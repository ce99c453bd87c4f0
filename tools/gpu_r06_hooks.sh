#!/bin/bash
# round 6: the pass-B gate / poisoned test build, the file-ingestion tests
set -o pipefail
mkdir -p gpurun_out/r06
timeout -k 10 900 python -u -m pytest tests/test_gpu_hooks.py::test_project_blocks_fused_vs_unfused tests/test_gpu_ingest.py -x -v -s --timeout 400 \
  --timeout-method thread > gpurun_out/r06/hooks_ingest.log 2>&1
rc=$?
tail -30 gpurun_out/r06/hooks_ingest.log
exit $rc
