#!/bin/bash
# round 6: IRL timing split (the small launches timed as "other") and the
# normest fused/split parity (mode 3 on CSR)
set -o pipefail
O=gpurun_out/r06/${TAG:-irl}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_hooks.py -k "normest or project_blocks" -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rep in 1 2; do
timeout -k 10 300 python bench.py --driver irl --workload circuit_1259 --no-cpu-baseline --steps 3 --warmup 1 > $O/irl.$rep.json 2> $O/irl.$rep.err || exit $?
python3 -c "
import json; i=json.load(open('$O/irl.$rep.json'))
print('irl %.2f solves/s split %s kernels %s' % (i['value'], i['time_split'], {k: round(v,3) for k,v in i['kernel_ms_per_solve'].items()}))"
done
