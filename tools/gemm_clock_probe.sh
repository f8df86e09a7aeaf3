#!/bin/bash
# Effective clock + wait split of encoder GEMM tile configs, one rocprofv3 PMC pass per
# (config, shape):  bash tools/gemm_clock_probe.sh "<configs>" "<shapes>"
# (round 3 default: the production two-stage kernel 10, its fill-only / compute-only builds 15 / 16,
# the loader / consumer kernel 17 and its halves 18 / 19 on rob_fc2)
R=${GRAFT_REPO_ROOT:-$(pwd)}
CFGS=${1:-"10 15 16 17 18 19"}
SHAPES=${2:-rob_fc2}
OUT=$R/gpurun_out/clockprobe
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for S in ${SHAPES//,/ }; do
  for C in $CFGS; do
    timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -f csv -d $OUT/${S}_c$C -o run -- python3 $R/tools/gemm_bench.py --configs $C --iters 30 --shapes $S > $OUT/${S}_c$C.log 2>&1 || exit 1
  done
done
