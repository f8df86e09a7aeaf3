#!/bin/bash
# Round-5 A/B: padded depthwise-tile pixels in the fused fronts (MMF_EDW_PAD) and the stem (MMF_SD_PAD)
# vs the unpadded builds: EfficientNet logits bit for bit + interleaved tower timings, every
# analyze_batch output bit for bit, the EfficientNet GPU tests, interleaved full-step timings.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; TAG=$1
OUT=$R/gpurun_out/$TAG; mkdir -p $OUT; cd $R
bash tools/effnet_ab_libs.sh $TAG 5 512 variants/pad0/libmmf_hip.so variants/edw8/libmmf_hip.so default || exit 1
MMF_HIP_LIB=$R/variants/pad0/libmmf_hip.so timeout -k 10 180 python3 tools/dump_step_outputs.py $OUT/var.npz 2>/dev/null || exit 1
timeout -k 10 180 python3 tools/dump_step_outputs.py $OUT/new.npz 2>/dev/null || exit 1
python3 tools/dump_step_outputs.py --cmp $OUT/var.npz $OUT/new.npz
timeout -k 10 400 python3 -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "effnet or image or stem" 2>&1 | tail -2 || exit 1
bash tools/lib_step_ab.sh 3 variants/pad0/libmmf_hip.so default 2>&1 | grep -v amdgpu.ids
