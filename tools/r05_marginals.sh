set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/r05m; mkdir -p $OUT; cd $R
timeout -k 10 300 python3 tools/step_ab.py "diag_skip=0" "diag_skip=14" "diag_skip=1" "diag_skip=15" "diag_skip=13" "diag_skip=11" "diag_skip=7" --rounds 5 --iters 15 > $OUT/marg.txt 2>&1 || exit 1
timeout -k 10 200 python3 tools/step_ab.py --what text "concurrent=1" "concurrent=0" --rounds 5 --iters 15 > $OUT/text.txt 2>&1 || exit 1
timeout -k 10 200 python3 tools/step_ab.py --what clip "concurrent=1" --rounds 5 --iters 15 > $OUT/clip.txt 2>&1 || exit 1
cat $OUT/*.txt | grep -v amdgpu.ids
