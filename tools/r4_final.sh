#!/bin/bash
# round-4 checkpoint on the GPU box: full -m gpu suite, default bench line, round profile (trace + PMC)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
TAG=${1:-r04}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/${TAG}_gputest.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > $O/${TAG}_bench.json 2> $O/${TAG}_bench.log || exit $?
timeout -k 10 600 bash tools/profile_round.sh ${TAG}prof || exit $?
