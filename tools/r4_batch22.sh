#!/bin/bash
# round-4 GPU batch 22: EfficientNet SE with 8 images per block (option se_group) -- bit identity,
# configs[2] workload A/B (fp16 and fp32 towers), whole step A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "se_image_groups or fp32_tower or effnet" -x -v --timeout 200 --timeout-method thread > $O/r4_se_test.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/effnet_bench.py --batch 512 --ab se_group=0 se_group=8 --rounds 5 > $O/r4_se_eff.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/effnet_bench.py --batch 512 --ab effnet_fp32=1,se_group=0 effnet_fp32=1,se_group=8 --rounds 3 > $O/r4_se_eff32.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/step_ab.py se_group=0 se_group=8 --rounds 4 > $O/r4_se_step.log 2>&1 || exit $?
