timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "fp32 or effnet" --timeout 200 --timeout-method thread > gpurun_out/t5.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_checkpoint.py -x -q -s -k "full_size" --timeout 200 --timeout-method thread > gpurun_out/t6.log 2>&1
bash tools/effnet32_prof.sh
