#!/bin/bash
# round 6: 'full' with pass B fused with the wide Gram (k_passb_wide):
# parity, then a same-box A/B of the full leg on the test build
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06/${TAG:-pbw}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_hooks.py tests/test_gpu_parity.py -k "full or wide or orth_err" -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rep in 1 2; do
for v in fused sep; do
  if [ $v = sep ]; then E="CAL_TEST_PASSB_WIDE_OFF=1"; else E=""; fi
  env CAL_LIBRARY=testhooks $E LEG_ORTH=full LEG_STEPS=14 LEG_REPS=1 timeout -k 10 300 python tools/leg_only.py > $O/full_$v.$rep.json 2> $O/full_$v.$rep.err || exit $?
  python3 -c "
import json; f=json.load(open('$O/full_$v.$rep.json'))[0]
print('%-5s full %.1f it/s gram %.3f apply %.3f' % ('$v', f['outer_iters_per_s'], f['kernel_ms_per_step']['gram'], f['kernel_ms_per_step']['apply']))"
done
done
LEG_ORTH=full LEG_STEPS=14 LEG_REPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/leg_only.py > $O/prof.json 2> $O/prof.err || exit $?
python3 tools/kstats.py $O/prof/run_kernel_stats.csv 8
