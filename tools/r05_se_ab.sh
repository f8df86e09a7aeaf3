#!/bin/bash
# Round-5 A/B of the SE kernel's load batching (pool partials 16 in flight, fc1 SE_FC1_U weights per
# output per step) against variants/sehead (previous commit) and variants/seu16: EfficientNet logits bit
# for bit + interleaved tower timings, fp32-tower / EfficientNet GPU tests, and se_kernel durations.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; TAG=$1
OUT=$R/gpurun_out/$TAG; mkdir -p $OUT; cd $R
bash tools/effnet_ab_libs.sh $TAG 5 512 variants/sehead/libmmf_hip.so variants/seu16/libmmf_hip.so default || exit 1
timeout -k 10 400 python3 -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "effnet or fp32 or se_" 2>&1 | tail -2 || exit 1
cd /tmp && export TMPDIR=/tmp
for L in sehead new; do
  if [ $L != new ]; then export MMF_HIP_LIB=$R/variants/$L/libmmf_hip.so; else unset MMF_HIP_LIB; fi
  timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/prof_$L -o run -- python3 $R/tools/effnet_bench.py --batch 256 --iters 10 > $OUT/prof_$L.log 2>&1 || exit 1
  python3 $R/tools/rocprof_summary.py $OUT/prof_$L/run_results.db > $OUT/prof_$L.txt 2>&1 || true
  echo "== $L"; grep -E "se_kernel|TOTAL" $OUT/prof_$L.txt
done
