#!/bin/bash
# PMC passes (one rocprofv3 run per counter group, as gfx950 requires) over a short command.
#   bash tools/pmc_passes.sh <tag> <command...>      e.g.  bash tools/pmc_passes.sh eff python3 tools/effnet_bench.py --iters 2
# Outputs gpurun_out/<tag>/p<N>/run_counter_collection.csv; summarise with tools/pmc_summary.py.
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
PASSES=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
  "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
  "FETCH_SIZE"
  "WRITE_SIZE"
)
i=0
for P in "${PASSES[@]}"; do
  i=$((i + 1))
  echo "pass $i: $P" >> $OUT/passes.log
  timeout -s KILL 120 rocprofv3 --pmc $P -f csv -d $OUT/p$i -o run -- "$@" > $OUT/p$i.log 2>&1 ||
    { echo "pass $i failed: exit $?" >> $OUT/passes.log; exit 1; }
done
echo done >> $OUT/passes.log
