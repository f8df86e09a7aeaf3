set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/r05se; mkdir -p $OUT; cd $R
for T in 0 1; do
MMF_HIP_LIB=$R/variants/base2/libmmf_hip.so timeout -k 10 120 python3 tools/effnet_dump.py $OUT/base$T.npy effnet_fp32=$T 2>/dev/null || exit 1
timeout -k 10 120 python3 tools/effnet_dump.py $OUT/new$T.npy effnet_fp32=$T 2>/dev/null || exit 1
python3 -c "import numpy as np;a=np.load('$OUT/base$T.npy');b=np.load('$OUT/new$T.npy');print('effnet_fp32=$T logits bit-identical to HEAD:', np.array_equal(a.view(np.uint32),b.view(np.uint32)))"
done
for r in 1 2 3; do
for L in variants/base2/libmmf_hip.so default; do
  if [ "$L" = default ]; then unset MMF_HIP_LIB; else export MMF_HIP_LIB=$R/$L; fi
  echo -n "$L B=256: "; timeout -k 10 120 python3 tools/effnet_bench.py --batch 256 --opt effnet_chunks=1 --iters 20 2>&1 | grep effnet || exit 1
done; done
unset MMF_HIP_LIB
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace -d $OUT/trace -o run -- python3 $R/tools/effnet_bench.py --batch 256 --iters 3 --opt effnet_chunks=1 > $OUT/trace.log 2>&1 || exit 1
python3 $R/tools/rocpd_summary.py $OUT/trace/run_results.db --grid --match se_kernel > $OUT/se.txt 2>&1
echo done
