#!/bin/bash
# Round-5 A/B of RoBERTa's add+LN rows per wave (MMF_LN_RPW): in-tree (2) vs variants/rpw1 (the
# previous kernel) and variants/rpw4: analyze_batch outputs bit for bit, text tests, text-only and
# full-step interleaved timings.   bash tools/r05_ln_ab.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; TAG=$1
OUT=$R/gpurun_out/$TAG; mkdir -p $OUT; cd $R
for V in rpw1 rpw4; do
  MMF_HIP_LIB=$R/variants/$V/libmmf_hip.so timeout -k 10 180 python3 tools/dump_step_outputs.py $OUT/$V.npz 2>/dev/null || exit 1
done
timeout -k 10 180 python3 tools/dump_step_outputs.py $OUT/new.npz 2>/dev/null || exit 1
python3 tools/dump_step_outputs.py --cmp $OUT/rpw1.npz $OUT/new.npz
python3 tools/dump_step_outputs.py --cmp $OUT/rpw1.npz $OUT/rpw4.npz
timeout -k 10 400 python3 -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "outlier or text or precise" 2>&1 | tail -2 || exit 1
for r in 1 2 3; do
  for L in variants/rpw1/libmmf_hip.so default variants/rpw4/libmmf_hip.so; do
    if [ "$L" = default ]; then unset MMF_HIP_LIB; else export MMF_HIP_LIB=$R/$L; fi
    echo -n "round $r $L text: "
    timeout -k 10 120 python3 tools/step_ab.py "concurrent=1" --what text --rounds 3 --iters 15 2>/dev/null | tail -1 || exit 1
  done
done
bash tools/lib_step_ab.sh 3 variants/rpw1/libmmf_hip.so default 2>&1 | grep -v amdgpu.ids
