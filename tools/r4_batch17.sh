#!/bin/bash
# round-4 GPU batch 17: split-K reduced by the last-arriving slice (option splitk_fix) -- bit identity,
# the existing split-K / small-batch tests, then B = 1 latency and step A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "splitk or small_batch or compact or batch_invariance" -x -v --timeout 200 --timeout-method thread > $O/r4_skf_test.log 2>&1 || exit $?
for r in 1 2 3; do
  for f in 0 1; do
    echo -n "round $r splitk_fix=$f: " >> $O/r4_skf_b1.log
    MMF_SPLITK_FIX=$f timeout -k 10 200 python3 tools/b1_latency.py --n 100 2>/dev/null | tail -1 >> $O/r4_skf_b1.log || exit 1
  done
done
timeout -k 10 300 python -u tools/step_ab.py splitk_fix=0 splitk_fix=1 --rounds 4 > $O/r4_skf_step.log 2>&1 || exit $?
