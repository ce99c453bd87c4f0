# kernel stats of the 'full' orth bench and the IRL (config 5 shape) bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-full_irl}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/full -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-legs --orth full > $O/full.json 2> $O/full.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/irl -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --driver irl --workload circuit_1259 > $O/irl.json 2> $O/irl.err || exit $?
for f in full irl; do
  python3 -c "
import json;d=json.load(open('$O/$f.json'));print('$f', d['metric'], round(d['value'],2), d.get('ms_per_step'))"
  python3 - "$O/$f/run_kernel_stats.csv" <<'PY'
import csv,sys
rows=sorted(csv.DictReader(open(sys.argv[1])), key=lambda r:-float(r['TotalDurationNs']))
tot=sum(float(r['TotalDurationNs']) for r in rows)
for r in rows[:12]: print('   %-60s %6s %9.1f us avg %5.1f%%'%(r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3, 100*float(r['TotalDurationNs'])/tot))
PY
done
