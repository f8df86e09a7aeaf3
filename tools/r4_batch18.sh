#!/bin/bash
# round-4 GPU batch 18: small batches enqueued by host threads per tower (option mt_enqueue)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "threaded_tower" -x -v --timeout 200 --timeout-method thread > $O/r4_mt_test.log 2>&1 || exit $?
for r in 1 2 3; do
  for f in 0 64; do
    echo -n "round $r mt_enqueue=$f: " >> $O/r4_mt_b1.log
    MMF_MT_ENQUEUE=$f timeout -k 10 200 python3 tools/b1_latency.py --n 100 2>/dev/null | tail -1 >> $O/r4_mt_b1.log || exit 1
  done
done
