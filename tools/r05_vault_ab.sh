#!/bin/bash
# Round-5 A/B of the vault kernels (similarities: several K chunks per barrier; top-k: one block of
# four waves per row) against variants/vhead (the previous commit): every analyze_batch output bit
# for bit, the vault GPU tests, and the two kernels' average durations from rocprofv3 --stats over
# the bench step.   bash tools/r05_vault_ab.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; TAG=$1
OUT=$R/gpurun_out/$TAG; mkdir -p $OUT; cd $R
MMF_HIP_LIB=$R/variants/${BASE:-vhead}/libmmf_hip.so timeout -k 10 180 python3 tools/dump_step_outputs.py $OUT/var.npz 2>/dev/null || exit 1
timeout -k 10 180 python3 tools/dump_step_outputs.py $OUT/new.npz 2>/dev/null || exit 1
python3 tools/dump_step_outputs.py --cmp $OUT/var.npz $OUT/new.npz
timeout -k 10 400 python3 -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "${K:-vault or analyze_pairs or fusion_training}" 2>&1 | tail -2 || exit 1
cd /tmp && export TMPDIR=/tmp
for L in ${LIBS:-vhead new}; do
  if [ $L != new ]; then export MMF_HIP_LIB=$R/variants/$L/libmmf_hip.so; else unset MMF_HIP_LIB; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof_$L -o run -- python3 $R/tools/step_ab.py "concurrent=1" --rounds 2 --iters 10 > $OUT/prof_$L.log 2>&1 || exit 1
  python3 $R/tools/rocprof_summary.py $OUT/prof_$L/run_results.db > $OUT/prof_$L.txt 2>&1 || true
  echo "== $L"; grep -E "${GREP:-vault|rowdot|fusion_kernel|attention_q1|text_heads|TOTAL}" $OUT/prof_$L.txt
done
