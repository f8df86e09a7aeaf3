set -o pipefail
T=gpurun_out/r06f; mkdir -p $T
timeout -k 10 200 python -u tools/dbg_eff_tmp.py > $T/dbg.txt 2>&1; rc=$?; cat $T/dbg.txt; exit $rc
