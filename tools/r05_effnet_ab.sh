#!/bin/bash
# EfficientNet-tower A/B of the in-tree library against variants/<base>: logits bit for bit + 5
# interleaved tower timings (B = 512), the EfficientNet / fp32 GPU tests, and per-kernel averages
# (rocprofv3 kernel trace over tools/effnet_bench.py, kernels matching GREP).
#   GREP="pw_kernel" bash tools/r05_effnet_ab.sh <tag> <base>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; TAG=$1; BASE=$2
OUT=$R/gpurun_out/$TAG; mkdir -p $OUT; cd $R
bash tools/effnet_ab_libs.sh $TAG 5 512 variants/$BASE/libmmf_hip.so default || exit 1
timeout -k 10 400 python3 -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "effnet or fp32 or se_" 2>&1 | tail -2 || exit 1
cd /tmp && export TMPDIR=/tmp
for L in $BASE new; do
  if [ $L != new ]; then export MMF_HIP_LIB=$R/variants/$L/libmmf_hip.so; else unset MMF_HIP_LIB; fi
  timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/prof_$L -o run -- python3 $R/tools/effnet_bench.py --batch 256 --iters 10 > $OUT/prof_$L.log 2>&1 || exit 1
  python3 $R/tools/rocprof_summary.py $OUT/prof_$L/run_results.db > $OUT/prof_$L.txt 2>&1 || true
  echo "== $L"; grep -E "${GREP:-TOTAL}|TOTAL" $OUT/prof_$L.txt
done
