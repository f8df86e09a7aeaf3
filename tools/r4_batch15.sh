#!/bin/bash
# round-4 GPU batch 15: tile order of the attention-epilogue launches only (option qkv_attn_gm)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
timeout -k 10 300 python -u tools/step_ab.py qkv_attn_gm=0 qkv_attn_gm=4 qkv_attn_gm=8 --rounds 5 --what text > $O/r4_qgm_text.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/step_ab.py qkv_attn_gm=0 qkv_attn_gm=4 qkv_attn_gm=8 --rounds 5 > $O/r4_qgm_step.log 2>&1 || exit $?
