# N>1 rehearsal of the overlapped matrix-powers schedule on one GPU: 2 ranks
# over the host-staged communicator, CAL_MPK_OVERLAP=1 (split) vs 0.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dist
for ov in 1 0; do
  CAL_MPK_OVERLAP=$ov timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 2 \
      --workload ${WL:-lap3d_120} --comm host > gpurun_out/dist/ov$ov.json 2> gpurun_out/dist/ov$ov.err || exit $?
done
echo done
