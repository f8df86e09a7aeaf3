#!/bin/bash
# round-4 GPU batch 10: attention in the RoBERTa QKV epilogue (option qkv_attn) -- bit identity, the
# profiler test, then interleaved step / text-only A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "qkv_attention_epilogue or batch_invariance or full_size_bench" tests/test_gpu_profiling.py -x -v --timeout 200 --timeout-method thread > $O/r4_qa_test.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/step_ab.py qkv_attn=0 qkv_attn=1 --rounds 5 > $O/r4_qa_step.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/step_ab.py qkv_attn=0 qkv_attn=1 --rounds 5 --what text > $O/r4_qa_text.log 2>&1 || exit $?
