#!/bin/bash
# round-4 GPU batch 5: fp32 tower deep-prefetch pw32m -- bit identity, tower A/B, kernel trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "fp32_tower" -x -v --timeout 200 --timeout-method thread > $O/r4_pw32_tests.log 2>&1 || exit $?
MMF_EFFNET_FP32=1 timeout -k 10 300 python -u tools/effnet_bench.py --batch 512 --iters 10 --ab pw32_mfma=1 pw32_mfma=2 --rounds 5 > $O/r4_pw32_ab.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
MMF_EFFNET_FP32=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/r4_f32prof2 -o run -- python3 $R/tools/effnet_bench.py --batch 512 --iters 5 > $O/r4_f32prof2.log 2>&1 || exit $?
