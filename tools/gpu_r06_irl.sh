#!/bin/bash
# round 6: the IRL with normest on its own stream: parity (async == sync norm,
# the restart tests, config 5 at full size) and two bench lines
set -o pipefail
O=gpurun_out/r06/${TAG:-irl}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_hooks.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_ingest.py -k "normest or restart or project_blocks or periodic or config5 or irl" -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rep in 1 2; do
timeout -k 10 300 python bench.py --driver irl --workload circuit_1259 --no-cpu-baseline --steps 3 --warmup 1 > $O/irl.$rep.json 2> $O/irl.$rep.err || exit $?
python3 -c "
import json; i=json.load(open('$O/irl.$rep.json'))
print('irl %.2f solves/s split %s kernels %s restarts %d' % (i['value'], i['time_split'], {k: round(v,3) for k,v in i['kernel_ms_per_solve'].items()}, i['num_restarts']))"
done
