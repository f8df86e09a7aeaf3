timeout -k 10 200 python -u tools/gemm_bench.py --configs 10,12,13,14 --iters 20 --shapes rob_o,rob_fc2,rob_qkv > gpurun_out/gb4.log 2>&1
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/ringpmc
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -f csv -d $R/gpurun_out/ringpmc/p1 -o run -- python3 $R/tools/gemm_bench.py --configs 10,12 --iters 10 --shapes rob_fc2 > $R/gpurun_out/ringpmc/p1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum -f csv -d $R/gpurun_out/ringpmc/p2 -o run -- python3 $R/tools/gemm_bench.py --configs 10,12 --iters 10 --shapes rob_fc2 > $R/gpurun_out/ringpmc/p2.log 2>&1
cd /tmp && timeout -s KILL 200 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/b1prof -o run -- python3 $R/tools/b1_latency.py --n 20 > $R/gpurun_out/b1prof.log 2>&1
