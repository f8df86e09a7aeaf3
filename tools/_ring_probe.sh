timeout -k 10 200 python -u tools/gemm_bench.py --configs 10,15,16,12,13,14 --iters 20 --shapes rob_o,rob_fc2,rob_qkv,txt_fc2 > gpurun_out/gb5.log 2>&1
