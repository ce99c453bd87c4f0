# A/B of the pair SpMV block size (CAL_PAIR_TB), bench at full size and at the 8-GPU per-rank size
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-tb_ab}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread -k "spmv or powers" > $O/pt.log 2>&1 || { tail -20 $O/pt.log; exit 1; }
CAL_PAIR_TB=1024 timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread -k "spmv or powers" > $O/pt512.log 2>&1 || { tail -20 $O/pt512.log; exit 1; }
tail -1 $O/pt512.log
for rep in 1 2; do
for tb in 512 1024; do
    for w in lap3d_215 lap3d_108; do
        CAL_PAIR_TB=$tb timeout -k 10 200 python bench.py --no-cpu-baseline --no-legs --workload $w --steps 40 > $O/b_${tb}_$w.json 2> $O/b_${tb}_$w.err || exit 1
        python -c "import json; d=json.load(open('$O/b_${tb}_$w.json')); print('tb', $tb, '$w', round(d['value'],1), round(d['spmv_avg_us'],2))"
    done
done
done
