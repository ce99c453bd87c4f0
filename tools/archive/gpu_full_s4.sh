# 'full' s = 4 parity (the (17, 4) row-apply shape), the restart tests, and
# the 'full' / restart results with the wide Gram kernel on (CAL_GRAM_AB=1)
# and off, compared
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/t3
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu -k "full_s4 or restarted or newton_full" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
grep -E "PASSED|FAILED|^E |passed|failed" $O/pytest.log | tail -10
CAL_GRAM_AB=1 timeout -k 10 200 python tools/gram_ab_lanczos.py ab1 2>&1 | tail -1 || exit $?
CAL_GRAM_AB=0 timeout -k 10 200 python tools/gram_ab_lanczos.py ab0 2>&1 | tail -1 || exit $?
python3 - <<'PY'
import numpy as np
a = np.load("gpurun_out/gram_ab_ab1.npz"); b = np.load("gpurun_out/gram_ab_ab0.npz")
print("T diff", np.max(np.abs(a["T"] - b["T"])), "rn diff", np.max(np.abs(a["rn"] - b["rn"])),
      "restarts", int(a["nres"]), int(b["nres"]))
PY
