#!/bin/bash
# rocprof kernel stats of the bench step (tower streams serialised) for several builds of libmmf_hip.so
#   bash tools/bench_prof_libs.sh <tag> lib1.so lib2.so ...   (lib "default" = the in-tree build)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export MMF_CONCURRENT=0
i=0
for L in "$@"; do
  i=$((i+1))
  if [ "$L" = default ]; then unset MMF_HIP_LIB; else export MMF_HIP_LIB=$R/$L; fi
  echo "t$i $L" >> $OUT/libs.txt
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/t$i -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-configs --no-profile > $OUT/t$i.log 2>&1 || exit 1
done
