#!/bin/bash
# round-4 GPU batch 8: full -m gpu suite on the current tree, then the RoBERTa-only last_q1 step A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r4_gputest2.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/step_ab.py last_q1=0 last_q1=1 --rounds 5 > $O/r4_q1_step2.log 2>&1 || exit $?
