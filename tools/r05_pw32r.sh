set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/r05p3; mkdir -p $OUT; cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 200 --timeout-method thread -k "fp32" 2>&1 | tail -3 || exit 1
timeout -k 10 300 python3 tools/effnet_bench.py --batch 512 --opt effnet_fp32=1 --ab pw32_mfma=2 pw32_mfma=4 pw32_mfma=5 --rounds 5 --iters 5 2>&1 | grep -v amdgpu.ids || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace -d $OUT/trace -o run -- python3 $R/tools/effnet_bench.py --batch 256 --iters 3 --opt effnet_chunks=1 effnet_fp32=1 pw32_mfma=5 > $OUT/trace.log 2>&1 || exit 1
python3 $R/tools/rocpd_summary.py $OUT/trace/run_results.db --grid --per 4 > $OUT/all.txt 2>&1
echo done
