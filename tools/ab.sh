#!/bin/bash
# A/B the exp/libmhmkc_*.so variants on the C2 bench (one GPU call). Stops at the first abnormal exit.
set -o pipefail
mkdir -p gpurun_out
for lib in exp/libmhmkc_*.so; do
  n=$(basename $lib .so)
  MHMKC_LIB=$PWD/$lib timeout -k 10 300 python bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline > gpurun_out/ab_$n.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "$n failed rc=$rc"; tail -5 gpurun_out/ab_$n.log; exit $rc; fi
  python - gpurun_out/ab_$n.log $n <<'PY'
import json, sys
j = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
st = {k: v for k, v in j["stages_ms_per_step"].items() if v > 0.05}
print(f'{sys.argv[2]:28s} {j["value"]/1e9:6.2f} G/s  {j["ms_per_step"]:7.2f} ms  {st}')
PY
done
