set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/b_head.json 2> gpurun_out/b_head.err && \
timeout -k 10 300 python bench.py --workload circuit_1259 --no-cpu-baseline > gpurun_out/b_circ.json 2> gpurun_out/b_circ.err && \
timeout -k 10 300 python bench.py --workload lap2d_3162 --no-cpu-baseline > gpurun_out/b_lap2d.json 2> gpurun_out/b_lap2d.err && \
timeout -k 10 400 python bench.py --workload circuit_1259 --driver irl > gpurun_out/b_irl.json 2> gpurun_out/b_irl.err
echo rc=$?
