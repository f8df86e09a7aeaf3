#!/bin/bash
# Counter attribution of the encoder GEMM K loop: the wait / issue / MFMA split
# and the effective clock, per kernel, on the isolated shapes (tools/gemm_bench.py) and on the
# bench step.  One rocprofv3 run per counter group (gfx950 slot limits: 8 SQ, 2 GRBM, 4 TCC).
#   bash tools/gemm_pmc.sh <tag>       -> gpurun_out/<tag>/{iso,step}/p<N>/run_counter_collection.csv
set -o pipefail
TAG=${1:-gemmpmc}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
PASSES=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
  "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum"
  "FETCH_SIZE"
  "WRITE_SIZE"
)
run_passes() {  # $1 = sub-dir, rest = command
  local D=$OUT/$1; shift
  mkdir -p $D
  local i=0
  for P in "${PASSES[@]}"; do
    i=$((i + 1))
    echo "pass $i: $P" >> $D/passes.log
    timeout -s KILL 150 rocprofv3 --pmc $P -f csv -d $D/p$i -o run -- "$@" > $D/p$i.log 2>&1 || { echo "pass $i failed rc=$?" >> $D/passes.log; return 1; }
  done
}
[ "${STEP_ONLY:-0}" = 1 ] || run_passes iso python3 $R/tools/gemm_bench.py --configs auto --iters 10 --shapes rob_qkv,rob_o,rob_fc1,rob_fc2,vit_fc2,sq4096 && \
run_passes step python3 $R/bench.py --steps 3 --warmup 2 --no-configs --no-per-sample --no-cpu-baseline --no-profile --no-e2e
echo done >> $OUT/passes.log
