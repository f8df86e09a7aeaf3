set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/r05o6; mkdir -p $OUT; cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 200 --timeout-method thread -k "tower_order" 2>&1 | tail -2 || exit 1
timeout -k 10 400 python3 tools/step_ab.py "after_text=12" "after_text=12,eff_split=1" "after_text=0" --rounds 6 --iters 15 > $OUT/order.txt 2>&1 || exit 1
grep -v amdgpu.ids $OUT/order.txt
