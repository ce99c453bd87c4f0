# Round 4 same-box A/B of the non-temporal Q stores (CAL_NT_OFF=1 turns them off), alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r04_nt_ab}
mkdir -p $O
for i in 1 2 3; do for v in off on; do
  if [ $v = off ]; then export CAL_NT_OFF=1; else unset CAL_NT_OFF; fi
  for nz in auto tsqr; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-legs --steps 30 --normalize $nz > $O/b_${v}_${nz}_$i.json 2> $O/b_${v}_${nz}_$i.err || exit 1
    python - $O/b_${v}_${nz}_$i.json $v $nz <<'PY'
import json,sys
d=json.load(open(sys.argv[1]))
print(sys.argv[2], sys.argv[3], round(d['value'],1), {k: round(v,3) for k,v in d['kernel_ms_per_step'].items()})
PY
  done
done; done
