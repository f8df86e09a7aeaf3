#!/bin/bash
# round-4 GPU batch 7: compact last-layer queries (option last_q1) -- parity suites, then step / CLIP / text A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py tests/test_gpu_checkpoint.py tests/test_gpu_outliers.py -x -q --timeout 300 --timeout-method thread > $O/r4_q1_tests.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/step_ab.py last_q1=0 last_q1=1 --rounds 5 > $O/r4_q1_step.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/step_ab.py last_q1=0 last_q1=1 --what clip --rounds 5 > $O/r4_q1_clip.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/step_ab.py last_q1=0 last_q1=1 --what text --rounds 5 > $O/r4_q1_text.log 2>&1 || exit $?
