#!/bin/bash
# direct-layout Gram probe, then the RCCL bench rehearsal
mkdir -p gpurun_out/direct
timeout -k 10 120 ./tools/direct_gram_probe > gpurun_out/direct/probe.json 2>&1 || { cat gpurun_out/direct/probe.json; exit 1; }
cat gpurun_out/direct/probe.json
bash tools/gpu_r05_rccl_bench.sh
