set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/r05q; mkdir -p $OUT; cd $R
for i in 1 2; do
for Q in 4 8; do
  GPU_MAX_HW_QUEUES=$Q timeout -k 10 300 python3 tools/step_ab.py "after_text=12" "after_text=0" --rounds 4 --iters 15 2>&1 | grep "ms/step" | sed "s/^/hwq=$Q /" || exit 1
  GPU_MAX_HW_QUEUES=$Q timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-configs --no-per-sample --no-e2e --no-profile > $OUT/bench_$Q.$i.json 2>$OUT/bench_$Q.$i.err || exit 1
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print('hwq=$Q bench', d['value'], d['ms_per_step'], d['hbm_resident']['value'])" $OUT/bench_$Q.$i.json
done; done
