#!/bin/bash
# round-4 GPU batch 6: fused fp32 fronts -- bit identity, fp32-tower parity tests, A/B, kernel trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "fp32" -v --timeout 300 --timeout-method thread > $O/r4_f32fuse_tests.log 2>&1 || exit $?
MMF_EFFNET_FP32=1 timeout -k 10 300 python -u tools/effnet_bench.py --batch 512 --iters 10 --ab fuse_expand32=0 fuse_expand32=1 --rounds 5 > $O/r4_f32fuse_ab.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
MMF_EFFNET_FP32=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/r4_f32prof3 -o run -- python3 $R/tools/effnet_bench.py --batch 512 --iters 5 > $O/r4_f32prof3.log 2>&1 || exit $?
