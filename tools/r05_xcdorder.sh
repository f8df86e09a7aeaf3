set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/r05x; mkdir -p $OUT; cd $R
timeout -k 10 300 python3 tools/step_ab.py --what text "gemm_group_m=0" "gemm_group_m=-1" "gemm_group_m=-2" "gemm_group_m=-4" --rounds 5 --iters 15 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 300 python3 tools/step_ab.py "gemm_group_m=0" "gemm_group_m=-1" "gemm_group_m=-2" --rounds 5 --iters 15 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 300 python3 tools/step_ab.py --what clip "gemm_group_m=0" "gemm_group_m=-1" "gemm_group_m=-2" --rounds 5 --iters 15 2>&1 | grep -v amdgpu.ids || exit 1
