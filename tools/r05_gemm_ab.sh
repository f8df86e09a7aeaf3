#!/bin/bash
# GEMM A/B of the in-tree library against variants/<base>: every analyze_batch output bit for bit, the
# GEMM / encoder GPU tests, interleaved text-only (configs[1]), CLIP (configs[3]) and full-step timings.
#   bash tools/r05_gemm_ab.sh <tag> <base>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; TAG=$1; BASE=$2
OUT=$R/gpurun_out/$TAG; mkdir -p $OUT; cd $R
MMF_HIP_LIB=$R/variants/$BASE/libmmf_hip.so timeout -k 10 180 python3 tools/dump_step_outputs.py $OUT/var.npz 2>/dev/null || exit 1
timeout -k 10 180 python3 tools/dump_step_outputs.py $OUT/new.npz 2>/dev/null || exit 1
python3 tools/dump_step_outputs.py --cmp $OUT/var.npz $OUT/new.npz
timeout -k 10 500 python3 -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "${K:-gemm or text or clip or parity}" 2>&1 | tail -2 || exit 1
for r in 1 2 3; do
  for L in variants/$BASE/libmmf_hip.so default; do
    if [ "$L" = default ]; then unset MMF_HIP_LIB; else export MMF_HIP_LIB=$R/$L; fi
    for W in text clip; do
      echo -n "round $r $L $W: "
      timeout -k 10 120 python3 tools/step_ab.py "concurrent=1" --what $W --rounds 3 --iters 15 2>/dev/null | tail -1 || exit 1
    done
  done
done
bash tools/lib_step_ab.sh 3 variants/$BASE/libmmf_hip.so default 2>&1 | grep -v amdgpu.ids
