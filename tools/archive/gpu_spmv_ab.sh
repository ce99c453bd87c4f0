# A/B of the CSR SpMV block order (CAL_SPMV_XCD), alternating, same box
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-spmv_ab}
mkdir -p $O
for rep in 1 2; do
  for x in 0 1; do
    for w in lap3d_215 circuit_1259; do
      CAL_SPMV_XCD=$x timeout -k 10 200 python tools/spmv_sweep.py --workload $w --format csr --reps 50 >> $O/spmv.jsonl 2>> $O/err.log || exit 1
    done
  done
done
python -c "
import json
for l in open('$O/spmv.jsonl'):
    d=json.loads(l); print(d['workload'], d['env'], round(d['mean_us'],1), round(d['gbps_mean']))"
