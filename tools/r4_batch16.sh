#!/bin/bash
# round-4 GPU batch 16: per-stream timeline of B = 1 analyze_batch calls
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O/r4_b1trace
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -f csv rocpd -d $O/r4_b1trace -o run -- python3 $R/tools/b1_trace.py --calls 40 > $O/r4_b1trace.log 2>&1 || exit $?
python3 $R/tools/b1_trace.py --report $O/r4_b1trace/run_results.db --last 2 > $O/r4_b1trace_report.txt 2>&1
rm -f $O/r4_b1trace/*.csv
