#!/bin/bash
# round-4 GPU batch 11: persistent tile order (gemm_group_m) re-measured with the attention epilogue
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
timeout -k 10 300 python -u tools/step_ab.py gemm_group_m=0 gemm_group_m=4 gemm_group_m=8 gemm_group_m=16 --rounds 4 --what text > $O/r4_gm_text.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/step_ab.py gemm_group_m=0 gemm_group_m=4 gemm_group_m=8 --rounds 4 > $O/r4_gm_step.log 2>&1 || exit $?
