#!/bin/bash
# One GPU call of the round (run from the repo root through gpurun):
#   tools/gpu_round.sh <tag> [pytest selection...]
# 1. the -m gpu suite (or the given selection) with a per-test limit, log under gpurun_out/<tag>/
# 2. a default bench.py line (skipped with NO_BENCH=1)
# Every GPU step has its own time limit and the script stops at the first failing step.
set -o pipefail
TAG=${1:-gpu}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
SEL=${@:-tests}
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 ${TEST_LIMIT:-1500} python -u -m pytest $SEL -m gpu -v -rA --timeout 600 --timeout-method thread \
    > $OUT/pytest.log 2>&1
  rc=$?
  tail -40 $OUT/pytest.log
  echo "pytest rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi  # (1 = test failures: the bench still runs)
fi
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 ${BENCH_LIMIT:-400} python -u bench.py ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err
  rc=$?
  tail -5 $OUT/bench.err
  echo "bench rc=$rc"
  exit $rc
fi
