set -o pipefail
T=gpurun_out/r06m; mkdir -p $T
timeout -k 10 600 python -u -m pytest tests/test_gpu_traps.py tests/test_gpu_outliers.py tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -k "trap or gamma or precise or outlier" > $T/pytest.log 2>&1
rc=$?; tail -3 $T/pytest.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/text_modes_bench.py --gamma 7 > $T/text_modes.txt 2>&1; rc=$?; cat $T/text_modes.txt; exit $rc
