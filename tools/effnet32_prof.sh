#!/bin/bash
# fp32 EfficientNet tower kernel breakdown (rocprofv3 stats) at B=256
set -e
mkdir -p gpurun_out/e32
cd /tmp && export TMPDIR=/tmp
MMF_EFFNET_FP32=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/e32/trace -o run -- \
  python3 $GRAFT_REPO_ROOT/tools/effnet_bench.py --iters 5 > $GRAFT_REPO_ROOT/gpurun_out/e32/bench.log 2>&1
