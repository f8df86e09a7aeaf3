#!/bin/bash
# Interleaved A/B of EfficientNet-tower builds (separate processes, ROUNDS rounds) + bit-identity
# of their logits against the first library:
#   bash tools/effnet_ab_libs.sh <tag> <rounds> <batch> lib1 lib2 ...   ("default" = in-tree build)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; ROUNDS=$2; B=$3; shift 3
mkdir -p $OUT
for L in "$@"; do
  if [ "$L" = default ]; then unset MMF_HIP_LIB; else export MMF_HIP_LIB=$R/$L; fi
  timeout -k 10 120 python3 $R/tools/effnet_dump.py $OUT/$(echo $L | tr / _).npy || exit 1
done
python3 - "$OUT" "$@" <<'PY' | tee $OUT/bitcmp.txt
import sys, numpy as np
out, libs = sys.argv[1], sys.argv[2:]
ref = np.load(f"{out}/{libs[0].replace('/', '_')}.npy")
for l in libs[1:]:
    a = np.load(f"{out}/{l.replace('/', '_')}.npy")
    print(l, "bit-identical" if np.array_equal(a.view(np.uint32), ref.view(np.uint32)) else f"DIFFERS max {np.abs(a-ref).max():.3e}")
PY
for r in $(seq $ROUNDS); do
  for L in "$@"; do
    if [ "$L" = default ]; then unset MMF_HIP_LIB; else export MMF_HIP_LIB=$R/$L; fi
    echo -n "$L: " >> $OUT/times.txt
    timeout -k 10 120 python3 $R/tools/effnet_bench.py --batch $B --iters 20 >> $OUT/times.txt 2>&1 || exit 1
  done
done
cat $OUT/times.txt
