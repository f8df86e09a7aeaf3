set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/r05s; mkdir -p $OUT; cd $R
MMF_HIP_LIB=$R/variants/base/libmmf_hip.so timeout -k 10 120 python3 tools/effnet_dump.py $OUT/base.npy effnet_fp32=1 pw32_mfma=2 2>/dev/null || exit 1
timeout -k 10 120 python3 tools/effnet_dump.py $OUT/new.npy effnet_fp32=1 2>/dev/null || exit 1
python3 -c "import numpy as np;a=np.load('$OUT/base.npy');b=np.load('$OUT/new.npy');print('fp32 tower logits bit-identical to the base build:', np.array_equal(a.view(np.uint32),b.view(np.uint32)))"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_checkpoint.py tests/test_gpu_outliers.py -m gpu -q -x --timeout 300 --timeout-method thread -k "fp32 or effnet" 2>&1 | tail -2 || exit 1
timeout -k 10 300 python3 tools/effnet_bench.py --batch 512 --opt effnet_fp32=1 --rounds 1 --iters 10 2>&1 | grep -v amdgpu.ids || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace -d $OUT/trace -o run -- python3 $R/tools/effnet_bench.py --batch 256 --iters 3 --opt effnet_chunks=1 effnet_fp32=1 > $OUT/trace.log 2>&1 || exit 1
python3 $R/tools/rocpd_summary.py $OUT/trace/run_results.db --per 4 --match 32 > $OUT/k32.txt 2>&1
python3 $R/tools/rocpd_summary.py $OUT/trace/run_results.db --per 4 --match stem > $OUT/stem.txt 2>&1
echo done
