#!/bin/bash
# Round-5 EfficientNet A/B batch (one gpurun call):
#   1. bit-identity of the tower's logits + interleaved timings, HEAD baseline vs in-tree build (B = 512)
#   2. kernel trace of one 256-image chunk (effnet_chunks = 1) -> per-queue idle gaps (tools/stream_gaps.py)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r05e}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
ROUNDS=${ROUNDS:-5}
bash tools/effnet_ab_libs.sh $TAG/ab $ROUNDS 512 variants/base/libmmf_hip.so default || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace -d $OUT/trace -o run -- python3 $R/tools/effnet_bench.py --batch 256 --iters 5 --opt effnet_chunks=1 > $OUT/trace.log 2>&1 || exit 1
python3 $R/tools/stream_gaps.py $OUT/trace/run_results.db --window-kernel gap_classifier > $OUT/gaps.txt 2>&1
python3 $R/tools/rocpd_summary.py $OUT/trace/run_results.db --per 6 > $OUT/kernels.txt 2>&1
rm -f $OUT/trace/*.db-journal
echo done
