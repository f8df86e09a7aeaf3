#!/bin/bash
# round-4 GPU batch 26: host pipeline depth (MMF_PIPE_SLOTS 2 vs 3) on the bench headline
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
for r in 1 2 3; do
  for n in 2 3; do
    echo -n "round $r slots=$n: " >> $O/r4_slots.log
    MMF_PIPE_SLOTS=$n timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 --no-configs --no-per-sample --no-e2e --no-cpu-baseline --no-profile 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['hbm_resident']['value'])" >> $O/r4_slots.log || exit 1
  done
done
