#!/bin/bash
# round-4 GPU batch 19: threaded tower enqueue (mt_enqueue) vs batch size, back-to-back steps
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
for b in 4 16 64 256; do
  echo "== batch $b" >> $O/r4_mt_batch.log
  timeout -k 10 300 python -u tools/step_ab.py mt_enqueue=0 mt_enqueue=256 --rounds 4 --batch $b 2>/dev/null | tail -3 >> $O/r4_mt_batch.log || exit 1
done
