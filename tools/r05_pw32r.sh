set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/r05p4; mkdir -p $OUT; cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 200 --timeout-method thread -k "fp32" 2>&1 | tail -2 || exit 1
timeout -k 10 300 python3 tools/effnet_bench.py --batch 512 --opt effnet_fp32=1 --ab pw32_mfma=3 pw32_mfma=4 pw32_mfma=5 --rounds 5 --iters 5 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 300 python3 tools/effnet_bench.py --batch 256 --opt effnet_fp32=1 effnet_chunks=1 --ab pw32_mfma=3 pw32_mfma=4 pw32_mfma=5 --rounds 5 --iters 5 2>&1 | grep -v amdgpu.ids || exit 1
