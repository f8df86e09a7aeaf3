#!/bin/bash
# round-4 GPU batch: guard / JPEG tests, producer-tile and CU-split A/Bs, fp32-tower kernel profile
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_outliers.py tests/test_gpu_jpeg.py -v -s --timeout 300 --timeout-method thread > $O/r4_guard.log 2>&1
rc=$?
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u tools/step_ab.py ln_prod256=0 ln_prod256=1 --what clip --rounds 5 > $O/r4_prod256_clip.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/step_ab.py ln_prod256=0 ln_prod256=1 --rounds 5 > $O/r4_prod256_step.log 2>&1 || exit $?
timeout -k 10 250 python -u tools/step_ab.py cu_split=0 cu_split=32 cu_split=48 cu_split=64 --rounds 4 > $O/r4_cusplit.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
MMF_EFFNET_FP32=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/r4_f32prof -o run -- python3 $R/tools/effnet_bench.py --batch 512 --iters 5 > $O/r4_f32prof.log 2>&1 || exit $?
