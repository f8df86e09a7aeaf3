#!/bin/bash
# round-4 GPU batch 3: GEMM-kind PMC passes on the bench step (no e2e line), EfficientNet B=512 kernel trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
STEP_ONLY=1 timeout -k 10 600 bash tools/gemm_pmc.sh r4_gemmpmc2 || exit $?
for p in $O/r4_gemmpmc2/step/p*/; do
  f=$(ls $p/*counter_collection.csv 2>/dev/null | head -1)
  [ -n "$f" ] && python3 tools/pmc_summary.py $f --match gemm_glds --top 20 > $p/summary.txt 2>&1
  rm -f $p/*.csv
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/r4_effprof -o run -- python3 $R/tools/effnet_bench.py --batch 512 --iters 5 > $O/r4_effprof.log 2>&1 || exit $?
