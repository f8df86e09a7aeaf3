#!/bin/bash
# round-4 GPU batch 4: descriptor LDS-DMA fills -- GEMM / parity tests, then a whole-step library A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm_wide.py tests/test_gpu_gemm_ring.py tests/test_gpu_kernels.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/r4_gldsbuf_tests.log 2>&1 || exit $?
timeout -k 10 900 bash tools/lib_step_ab.sh 3 default variants/glds_addr/libmmf_hip.so > $O/r4_gldsbuf_ab.log 2>&1 || exit $?
