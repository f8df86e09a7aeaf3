set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/r05o4; mkdir -p $OUT; cd $R
timeout -k 10 400 python3 tools/step_ab.py "after_text=0" "after_text=12" "after_text=12,after_layer=11" "after_text=12,after_layer=10" "after_text=12,after_layer=8" "after_text=14,after_layer=11" --rounds 6 --iters 15 > $OUT/order.txt 2>&1 || exit 1
grep -v amdgpu.ids $OUT/order.txt
