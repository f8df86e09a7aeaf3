#!/bin/bash
# round-4 GPU batch 9: 4-wave 256x192 tiles (config 21) -- bit identity, then isolated shapes vs configs 10 / 11
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm_wide.py -x -q --timeout 120 --timeout-method thread > $O/r4_w4_test.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/gemm_bench.py --configs auto,10,11,21 --iters 20 \
  --shapes rob_qkv,rob_o,rob_fc1,rob_fc2,vit_qkv,vit_fc2,txt_fc1,sq4096 > $O/r4_w4_bench.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/step_ab.py gemm_w4=0 gemm_w4=1 --rounds 4 > $O/r4_w4_step.log 2>&1 || exit $?
