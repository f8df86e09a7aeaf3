#!/bin/bash
# round-4 GPU batch 21: result copies on their own stream (MMF_D2H_STREAM) -- bench headline A/B,
# interleaved separate processes
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
for r in 1 2 3; do
  for f in 0 1; do
    echo -n "round $r d2h_stream=$f: " >> $O/r4_d2h.log
    MMF_D2H_STREAM=$f timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 --no-configs --no-per-sample --no-e2e --no-cpu-baseline --no-profile 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['hbm_resident']['value'])" >> $O/r4_d2h.log || exit 1
  done
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_api.py -x -q --timeout 200 --timeout-method thread > $O/r4_d2h_api.log 2>&1 || exit $?
