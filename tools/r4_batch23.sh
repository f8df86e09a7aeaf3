#!/bin/bash
# round-4 GPU batch 23: split-K only for deep K (option splitk_min_k) -- B = 1 latency and the step
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
for r in 1 2 3; do
  for f in 0 1024 2048; do
    echo -n "round $r splitk_min_k=$f: " >> $O/r4_skmin_b1.log
    MMF_SPLITK_MIN_K=$f timeout -k 10 200 python3 tools/b1_latency.py --n 100 2>/dev/null | tail -1 >> $O/r4_skmin_b1.log || exit 1
  done
done
timeout -k 10 300 python -u tools/step_ab.py splitk_min_k=0 splitk_min_k=1024 --rounds 4 > $O/r4_skmin_step.log 2>&1 || exit $?
