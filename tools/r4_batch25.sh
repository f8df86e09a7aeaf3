#!/bin/bash
# round-4 GPU batch 25: B = 1 latency with 4 (HIP default) vs 8 hardware queues per process
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
for r in 1 2 3; do
  for q in 4 8; do
    echo -n "round $r hw_queues=$q: " >> $O/r4_hwq_b1.log
    GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python3 tools/b1_latency.py --n 100 2>/dev/null | tail -1 >> $O/r4_hwq_b1.log || exit 1
  done
done
