#!/bin/bash
# Library A/B (run on the GPU box from the repo root): tools/knob_ab.py at k = $1 with the tree's library and with
# exp/libmhmkc_$2.so (MHMKC_LIB), alternated twice; then the variant's parity on the oracle tests. Logs under gpurun_out/.
set -o pipefail
k=$1; v=$2; P=gpurun_out/ab_${v}_k${k}
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 200 python3 -u tools/knob_ab.py $k "" > $P.default$i.log 2>&1 || { echo "default $i failed"; tail -3 $P.default$i.log; exit 1; }
  MHMKC_LIB=exp/libmhmkc_$v.so timeout -k 10 200 python3 -u tools/knob_ab.py $k "" > $P.$v$i.log 2>&1 || { echo "$v $i failed"; tail -3 $P.$v$i.log; exit 1; }
done
grep -h round $P.*.log
