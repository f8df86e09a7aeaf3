set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/r05o7; mkdir -p $OUT; cd $R
timeout -k 10 500 python3 tools/step_ab.py "eff_wait_block=0" "eff_wait_block=3" "eff_wait_block=5" "eff_wait_block=8" "eff_wait_block=11" "eff_wait_block=14" --rounds 5 --iters 15 > $OUT/order.txt 2>&1 || exit 1
grep -v amdgpu.ids $OUT/order.txt
