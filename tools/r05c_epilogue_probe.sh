# round-5 probe: 256x256 vs 256x192 tiles and the epilogue's store share (variants/skip*: a
# quarter / all of the fp16 epilogue stores dropped by the buffer descriptor; measurement only)
set -o pipefail
mkdir -p gpurun_out/r05c
for v in prod skip2 skip8; do
  if [ $v = prod ]; then unset MMF_HIP_LIB; else export MMF_HIP_LIB=variants/$v/libmmf_hip.so; fi
  timeout -k 10 240 python tools/gemm_bench.py --configs 10,11 --iters 30 \
    --shapes rob_qkv,rob_fc1,vit_qkv,vit_fc1,txt_qkv,txt_fc1,rob_o,rob_fc2 > gpurun_out/r05c/bench_$v.txt 2>&1 || exit $?
done
tail -n 9 gpurun_out/r05c/bench_*.txt
