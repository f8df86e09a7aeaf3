#!/bin/bash
# Round-5 A/B batch: the in-tree library vs variants/$VAR (a build of the same tree with one change
# reverted): every analyze_batch output compared bit for bit (tools/dump_step_outputs.py), a GPU test
# selection, and interleaved full-step timings (tools/lib_step_ab.sh).   bash tools/r05_batch.sh <tag> <variant> [pytest -k]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; TAG=$1; VAR=$2; K=${3:-vault}
OUT=$R/gpurun_out/$TAG; mkdir -p $OUT; cd $R
MMF_HIP_LIB=$R/variants/$VAR/libmmf_hip.so timeout -k 10 180 python3 tools/dump_step_outputs.py $OUT/var.npz 2>/dev/null || exit 1
timeout -k 10 180 python3 tools/dump_step_outputs.py $OUT/new.npz 2>/dev/null || exit 1
python3 tools/dump_step_outputs.py --cmp $OUT/var.npz $OUT/new.npz
timeout -k 10 400 python3 -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "$K" 2>&1 | tail -2 || exit 1
bash tools/lib_step_ab.sh 3 variants/$VAR/libmmf_hip.so default 2>&1 | grep -v amdgpu.ids
