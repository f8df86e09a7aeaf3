set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/r05f2; mkdir -p $OUT; cd $R
timeout -k 10 300 python3 tools/effnet_bench.py --batch 512 --ab fuse_expand_cin=64 fuse_expand_cin=96 --rounds 5 --iters 10 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 300 python3 tools/effnet_bench.py --batch 256 --opt effnet_chunks=1 --ab fuse_expand_cin=64 fuse_expand_cin=96 --rounds 5 --iters 10 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 400 python3 tools/step_ab.py "fuse_expand_cin=64" "fuse_expand_cin=96" --rounds 6 --iters 15 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kernels.py tests/test_gpu_checkpoint.py -m gpu -q -x --timeout 300 --timeout-method thread -k "effnet or fused or expand or calibration" 2>&1 | tail -3
