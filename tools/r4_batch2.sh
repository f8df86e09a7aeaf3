#!/bin/bash
# round-4 GPU batch 2: dominating-channel guard test, CU-split mask layouts, GEMM-kind PMC passes on the step
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_outliers.py -k dominating -v -s --timeout 300 --timeout-method thread > $O/r4_guard2.log 2>&1
rc=$?
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/step_ab.py cu_split=0 cu_split=32,cu_split_layout=1 cu_split=32,cu_split_layout=2 cu_split=64,cu_split_layout=1 cu_split=64,cu_split_layout=2 --rounds 3 > $O/r4_cusplit2.log 2>&1 || exit $?
STEP_ONLY=1 timeout -k 10 600 bash tools/gemm_pmc.sh r4_gemmpmc || exit $?
# reduce the PMC csvs on the box (raw files exceed gpurun's 64 MiB copy-back)
for p in $O/r4_gemmpmc/step/p*/; do
  f=$(ls $p/*counter_collection.csv 2>/dev/null | head -1)
  [ -n "$f" ] && python3 tools/pmc_summary.py $f --match gemm_glds --top 20 > $p/summary.txt 2>&1
  rm -f $p/*.csv
done
