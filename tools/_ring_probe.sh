timeout -k 10 200 python -u tools/gemm_bench.py --configs 10,15,16,17,18,19 --iters 20 --shapes rob_o,rob_fc2,rob_qkv,txt_fc2 > gpurun_out/gb7.log 2>&1
