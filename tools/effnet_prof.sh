#!/bin/bash
# rocprof kernel stats of the effnet tower alone, for option variants given as env assignments
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for V in "$@"; do
  i=$((i+1))
  export $V
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $OUT/t$i -o run -- python3 $R/tools/effnet_bench.py --iters 5 > $OUT/t$i.log 2>&1 || exit 1
done
