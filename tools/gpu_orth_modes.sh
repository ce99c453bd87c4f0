cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/orth
for o in local full periodic selective; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --orth $o --steps 15 > gpurun_out/orth/$o.json 2> gpurun_out/orth/$o.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/orth/$o.json'));print('$o', round(d['value'],1), d['ms_per_step'], d['kernel_ms_per_step'], d['reorth_passes'])"
done
