#!/bin/bash
# round-4 GPU batch 20: split-K on/off for the skinny GEMMs at B = 1 (latency) and in the step
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
for r in 1 2 3; do
  for f in 1 0; do
    echo -n "round $r gemm_splitk=$f: " >> $O/r4_sk_b1.log
    MMF_GEMM_SPLITK=$f timeout -k 10 200 python3 tools/b1_latency.py --n 100 2>/dev/null | tail -1 >> $O/r4_sk_b1.log || exit 1
  done
done
timeout -k 10 300 python -u tools/step_ab.py gemm_splitk=1 gemm_splitk=0 --rounds 4 > $O/r4_sk_step.log 2>&1 || exit $?
