#!/bin/bash
# tile-queue GEMMs (option gemm_tq): parity, then interleaved step / text / CLIP A/B
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "tile_queue or threaded_tower or qkv_attention or full_size_bench" > gpurun_out/r4b28_tests.log 2>&1 &&
timeout -k 10 240 python -u tools/step_ab.py gemm_tq=0 gemm_tq=1 --rounds 5 --iters 20 > gpurun_out/r4b28_step.txt 2>&1 &&
timeout -k 10 200 python -u tools/step_ab.py gemm_tq=0 gemm_tq=1 --what text --rounds 5 --iters 20 > gpurun_out/r4b28_text.txt 2>&1 &&
timeout -k 10 200 python -u tools/step_ab.py gemm_tq=0 gemm_tq=1 --what clip --rounds 5 --iters 20 > gpurun_out/r4b28_clip.txt 2>&1
