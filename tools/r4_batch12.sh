#!/bin/bash
# round-4 GPU batch 12: attention epilogue with K / V fragment reads shared by a wave's two query
# tiles (in-tree lib) vs the first version (variants/qa_v1) -- bit identity, then library A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "qkv_attention_epilogue" -x -q --timeout 200 --timeout-method thread > $O/r4_qa2_test.log 2>&1 || exit $?
for r in 1 2 3; do
  for L in default variants/qa_v1/libmmf_hip.so; do
    if [ "$L" = default ]; then unset MMF_HIP_LIB; else export MMF_HIP_LIB=$R/$L; fi
    echo -n "round $r $L text: " >> $O/r4_qa2_ab.log
    timeout -k 10 120 python3 $R/tools/step_ab.py "qkv_attn=1" --rounds 3 --what text 2>/dev/null | tail -1 >> $O/r4_qa2_ab.log || exit 1
    echo -n "round $r $L step: " >> $O/r4_qa2_ab.log
    timeout -k 10 120 python3 $R/tools/step_ab.py "qkv_attn=1" --rounds 3 2>/dev/null | tail -1 >> $O/r4_qa2_ab.log || exit 1
  done
done
