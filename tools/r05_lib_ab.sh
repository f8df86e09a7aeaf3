#!/bin/bash
# Round-5 A/B of the in-tree library against variants/<variant> (e.g. a build of the previous commit):
# EfficientNet logits bit for bit + interleaved tower timings (B = 512), every analyze_batch output
# bit for bit, a GPU test selection, interleaved full-step timings.
#   bash tools/r05_lib_ab.sh <tag> <variant> [pytest -k expression]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; TAG=$1; VAR=$2; K=${3:-effnet}
OUT=$R/gpurun_out/$TAG; mkdir -p $OUT; cd $R
bash tools/effnet_ab_libs.sh $TAG 5 512 variants/$VAR/libmmf_hip.so default || exit 1
MMF_HIP_LIB=$R/variants/$VAR/libmmf_hip.so timeout -k 10 180 python3 tools/dump_step_outputs.py $OUT/var.npz 2>/dev/null || exit 1
timeout -k 10 180 python3 tools/dump_step_outputs.py $OUT/new.npz 2>/dev/null || exit 1
python3 tools/dump_step_outputs.py --cmp $OUT/var.npz $OUT/new.npz
timeout -k 10 500 python3 -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "$K" 2>&1 | tail -2 || exit 1
bash tools/lib_step_ab.sh 3 variants/$VAR/libmmf_hip.so default 2>&1 | grep -v amdgpu.ids
