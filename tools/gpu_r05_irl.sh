# Round 5: the IRL driver (BASELINE config 5 stand-in) line and its kernel trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r05_irl}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload circuit_1259 --driver irl --no-cpu-baseline > $O/irl.json 2> $O/irl.err
echo "irl rc=$?"
python3 -c "import json;d=json.load(open('$O/irl.json'));print(round(d['value'],2), d['roofline']['kernel_class'], round(d['roofline']['achieved']), d['time_split'], d['kernel_ms_per_solve'])"
