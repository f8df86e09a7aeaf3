#!/bin/bash
# Full-step A/B of several builds of libmmf_hip.so: HBM-resident B=256 analyze step, one process per
# (round, library), libraries interleaved over rounds.   bash tools/lib_step_ab.sh <rounds> lib1 lib2 ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
N=$1; shift
for r in $(seq 1 $N); do
  for L in "$@"; do
    if [ "$L" = default ]; then unset MMF_HIP_LIB; else export MMF_HIP_LIB=$R/$L; fi
    echo -n "round $r $L: "
    timeout -k 10 120 python3 $R/tools/step_ab.py "concurrent=1" --rounds 3 --iters 15 2>/dev/null | tail -1 || exit 1
  done
done
