#!/bin/bash
# round-4 GPU batch 24: how the bench's H2D / D2H copies execute (SDMA engine or blit kernels)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O/r4_copytrace
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -f csv -d $O/r4_copytrace -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-configs --no-per-sample --no-e2e --no-cpu-baseline --no-profile > $O/r4_copytrace.log 2>&1 || exit $?
ls $O/r4_copytrace > $O/r4_copytrace_files.txt
head -5 $O/r4_copytrace/run_memory_copy_stats.csv > $O/r4_copytrace_memstats.txt 2>&1 || true
grep -i "copy\|fill" $O/r4_copytrace/run_kernel_stats.csv > $O/r4_copytrace_copykernels.txt 2>&1 || true
python3 - <<'PY' > $O/r4_copytrace_summary.txt 2>&1 || true
import csv, collections, os
d = os.environ.get("O", "") or "."
PY
rm -f $O/r4_copytrace/run_kernel_trace.csv
