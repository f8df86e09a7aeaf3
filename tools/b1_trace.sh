cd /tmp && export TMPDIR=/tmp
MMF_CONCURRENT=1 timeout -s KILL 200 rocprofv3 --kernel-trace -f csv -d $GRAFT_REPO_ROOT/gpurun_out/b1prof2 -o run -- python3 $GRAFT_REPO_ROOT/tools/b1_latency.py --n 20 > $GRAFT_REPO_ROOT/gpurun_out/b1prof2.log 2>&1
