#!/bin/bash
# tile-queue GEMMs with one counter per 256-B line: parity, then interleaved text-only / step A/B
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "tile_queue" > gpurun_out/r4b31_tests.log 2>&1 &&
timeout -k 10 200 python -u tools/step_ab.py gemm_tq=0 gemm_tq=1 --what text --rounds 5 --iters 20 > gpurun_out/r4b31_text.txt 2>&1 &&
timeout -k 10 240 python -u tools/step_ab.py gemm_tq=0 gemm_tq=1 --rounds 5 --iters 20 > gpurun_out/r4b31_step.txt 2>&1
