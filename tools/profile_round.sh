#!/bin/bash
# Round-end profiling on the GPU box (run from the repo root through gpurun):
#   1. kernel trace + stats of the bench command (sequential tower streams so every kernel's
#      duration is its own, comparable with bench.py's event timing)
#   2. two separate PMC passes (FETCH_SIZE, WRITE_SIZE -- they do not fit one pass on gfx950)
# Outputs under gpurun_out/<tag>/ ; summarise with tools/rocprof_summary.py / tools/pmc_traffic.py.
set -eo pipefail
TAG=${1:-prof}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export MMF_CONCURRENT=0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv rocpd -d $OUT/trace -o run -- \
  python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-configs --no-per-sample --no-e2e > $OUT/bench_trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -f csv -d $OUT/pmc_fetch -o run -- \
  python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-configs --no-per-sample --no-e2e > $OUT/bench_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -f csv -d $OUT/pmc_write -o run -- \
  python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-configs --no-per-sample --no-e2e > $OUT/bench_write.log 2>&1
# reduce on the box (raw PMC csvs can pass gpurun's 64 MiB copy-back)
python3 $R/tools/rocprof_summary.py $OUT/trace/run_results.db > $OUT/steady_state_kernels.txt 2>&1 || true
python3 $R/tools/pmc_traffic.py $OUT/pmc_fetch/run_counter_collection.csv $OUT/pmc_write/run_counter_collection.csv \
  --symbol 'gemm_glds_kernel<256, 192, 4, 2, 0, true, 0, 0>' --json $OUT/pmc_traffic.json > $OUT/pmc_traffic.txt 2>&1 || true
rm -f $OUT/pmc_fetch/*.csv $OUT/pmc_write/*.csv
echo done > $OUT/ok
