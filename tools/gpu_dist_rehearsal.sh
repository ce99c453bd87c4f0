# N>1 rehearsal on one GPU: 2 ranks over the host-staged (gloo) communicator,
# CA matrix powers (depth 8) vs one halo exchange per SpMV (depth 1).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dist
for d in 8 1; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 2 --workload ${WL:-lap3d_120} --comm host \
      --mpk-depth $d > gpurun_out/dist/d$d.json 2> gpurun_out/dist/d$d.err || exit $?
done
echo done
