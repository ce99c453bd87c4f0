# parity tests touching the wide Gram + 'full' orth bench + diagnostics-on run
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-gram}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -m gpu \
    -k "full or gram or wide or orth or selective or periodic" > $O/pt.log 2>&1 && \
timeout -k 10 200 python bench.py --orth full --no-cpu-baseline --no-legs > $O/full.json 2> $O/full.err && \
timeout -k 10 200 python tools/diag_only.py > $O/diag.json 2> $O/diag.err
rc=$?
tail -2 $O/pt.log
python -c "import json; d=json.load(open('$O/full.json')); print('full', round(d['value'],1), d['kernel_ms_per_step'] if 'kernel_ms_per_step' in d else '')"
cat $O/diag.json
exit $rc
