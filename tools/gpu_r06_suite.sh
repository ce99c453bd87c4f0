#!/bin/bash
# round 6: the GPU suite once on the production library, then once on the
# NaN-poisoned test build (CAL_LIBRARY=testhooks: every scratch buffer NaN
# when allocated, the block-orthogonalisation coefficient scratch NaN before
# each block), then smoke
set -o pipefail
O=gpurun_out/r06/${TAG:-suite}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_prod.log 2>&1 || { tail -40 $O/pytest_prod.log; exit 1; }
tail -2 $O/pytest_prod.log
CAL_LIBRARY=testhooks timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_poisoned.log 2>&1 || { tail -40 $O/pytest_poisoned.log; exit 1; }
tail -2 $O/pytest_poisoned.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log
