#!/bin/bash
mkdir -p gpurun_out/direct
timeout -k 10 120 ./tools/direct_gram_probe > gpurun_out/direct/probe2.json 2>&1; rc=$?
cat gpurun_out/direct/probe2.json; exit $rc
