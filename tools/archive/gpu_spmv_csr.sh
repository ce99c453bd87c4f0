# CSR SpMV timing (lap3d_215 and the circuit stand-in) and the IRL bench line
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-csr}
mkdir -p $O
for w in lap3d_215 circuit_1259; do
    timeout -k 10 200 python tools/spmv_sweep.py --workload $w --format csr --reps 50 >> $O/spmv.jsonl 2> $O/spmv_$w.err || exit 1
done
cat $O/spmv.jsonl
if [ -n "$IRL" ]; then
    timeout -k 10 400 python bench.py --workload circuit_1259 --driver irl --no-cpu-baseline > $O/irl.json 2> $O/irl.err || exit 1
    python -c "import json;d=json.load(open('$O/irl.json'));print('irl', d['value'], d['unit'], {k: d[k] for k in d if 'spmv' in k})"
fi
