# A/B of the gram_lds grid cap (CAL_GRAM_CAP) on the 'full' orth bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-gram_cap}
mkdir -p $O
for rep in 1 2; do
for cap in 2048 1536 1024 768; do
  CAL_GRAM_CAP=$cap timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-legs --orth full --steps 20 > $O/full_$cap.$rep.json 2> $O/full_$cap.$rep.err || exit $?
  python3 -c "import json;d=json.load(open('$O/full_$cap.$rep.json'));print('cap $cap rep $rep', round(d['value'],2))"
done
done
export TMPDIR=/tmp
cd /tmp
for cap in 2048 768; do
CAL_GRAM_CAP=$cap timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$cap -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-legs --orth full --steps 10 > /dev/null 2>&1 || exit $?
python3 - "$O/prof_$cap/run_kernel_stats.csv" <<'PY'
import csv,sys
rows=sorted(csv.DictReader(open(sys.argv[1])), key=lambda r:-float(r['TotalDurationNs']))
for r in rows[:6]: print('   %-60s %6s %9.1f us avg'%(r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3))
PY
done
