set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/r05o8; mkdir -p $OUT; cd $R
timeout -k 10 500 python3 tools/step_ab.py "text_after_vit=0" "text_after_vit=1" "text_after_vit=2" "text_after_vit=4" "text_after_vit=6" --rounds 5 --iters 15 > $OUT/order.txt 2>&1 || exit 1
grep -v amdgpu.ids $OUT/order.txt
