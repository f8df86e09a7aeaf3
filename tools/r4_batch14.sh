#!/bin/bash
# round-4 GPU batch 14: GEMM-kind PMC passes on the bench step with the attention-epilogue kind
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
STEP_ONLY=1 timeout -k 10 600 bash tools/gemm_pmc.sh r4_gemmpmc3 || exit $?
for p in $O/r4_gemmpmc3/step/p*/; do
  f=$(ls $p/*counter_collection.csv 2>/dev/null | head -1)
  [ -n "$f" ] && python3 tools/pmc_summary.py $f --match gemm_glds --top 20 > $p/summary.txt 2>&1
  rm -f $p/*.csv
done
