#!/bin/bash
# tools/ab.sh at another k: K=63 bash tools/ab_k.sh (each exp/libmhmkc_*.so, twice, C2 reads)
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
for lib in exp/libmhmkc_*.so; do
  n=$(basename $lib .so)
  MHMKC_LIB=$PWD/$lib timeout -k 10 300 python bench.py --k ${K:-63} --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --h2d-steps 0 --no-kmermap > gpurun_out/abk_$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/abk_$n.log; exit 1; }
  python - gpurun_out/abk_$n.log $n <<'PY'
import json, sys
j = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
st = {k: v for k, v in j["stages_ms_per_step"].items() if v > 0.05}
print(f'{sys.argv[2]:28s} k={j["config"]["k"]} {j["ms_per_step"]:7.2f} ms  {st}')
PY
done
done
