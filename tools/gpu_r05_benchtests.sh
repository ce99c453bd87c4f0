#!/bin/bash
mkdir -p gpurun_out/benchtests
timeout -k 10 900 python -u -m pytest tests/test_gpu_bench.py -x -v --timeout 400 --timeout-method thread > gpurun_out/benchtests/pytest.log 2>&1
rc=$?; tail -12 gpurun_out/benchtests/pytest.log; exit $rc
