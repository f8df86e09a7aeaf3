set -o pipefail
T=gpurun_out/r06j; mkdir -p $T
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_traps.py tests/test_gpu_outliers.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "gemm or trap or gamma or precise or outlier or golden" > $T/pytest.log 2>&1
rc=$?; tail -3 $T/pytest.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for L in variants/base/libmmf_hip.so default; do
    if [ "$L" = default ]; then unset MMF_HIP_LIB; else export MMF_HIP_LIB=$PWD/$L; fi
    echo "== round $r $L" >> $T/gemm_bench.txt
    timeout -k 10 200 python -u tools/gemm_bench.py --configs 10,11 --rounds 2 --iters 20 --shapes rob_qkv,rob_o,rob_fc1,rob_fc2,patch,vit_fc2 >> $T/gemm_bench.txt 2>&1 || exit 1
  done
done
unset MMF_HIP_LIB
cat $T/gemm_bench.txt
bash tools/lib_step_ab.sh 3 variants/base/libmmf_hip.so default > $T/step_ab.txt 2>&1; rc=$?; cat $T/step_ab.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/text_modes_bench.py --gamma 7 > $T/text_modes.txt 2>&1; rc=$?; cat $T/text_modes.txt; exit $rc
