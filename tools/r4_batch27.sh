#!/bin/bash
# EfficientNet PMC passes on the round-4 tree: B = 256 one chunk (round 3's setting) and B = 512 two chunks (configs[2])
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
timeout -k 10 180 python3 tools/effnet_bench.py --batch 512 --iters 20 > gpurun_out/eff_time.txt 2>&1 &&
timeout -k 10 700 bash tools/pmc_passes.sh eff256 python3 $R/tools/effnet_bench.py --batch 256 --iters 2 --opt effnet_chunks=1 &&
timeout -k 10 700 bash tools/pmc_passes.sh eff512 python3 $R/tools/effnet_bench.py --batch 512 --iters 2 &&
python3 tools/effnet_pmc_report.py gpurun_out/eff256 --images 768 > gpurun_out/eff256_report.txt &&
python3 tools/effnet_pmc_report.py gpurun_out/eff512 --images 1536 > gpurun_out/eff512_report.txt
