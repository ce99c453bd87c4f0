set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r05_spread gpurun_out/r05_grp
timeout -k 10 200 ./tools/gram_rows_probe > gpurun_out/r05_grp/probe.json || exit $?
timeout -k 10 300 python tools/restart_spread_dev.py 0 32 > gpurun_out/r05_spread/base.txt || exit $?
CAL_LIBRARY=variant_g0 timeout -k 10 300 python tools/restart_spread_dev.py 0 32 > gpurun_out/r05_spread/g0.txt
