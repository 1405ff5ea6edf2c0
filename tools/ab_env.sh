#!/bin/bash
# A/B of environment / library variants on the C2 bench in one GPU call. Each argument is
#   name|ENV=V ENV2=V2   (MHMKC_LIB=exp/... selects a library variant)
# Stops at the first abnormal exit.
set -o pipefail
mkdir -p gpurun_out
for spec in "$@"; do
  n=${spec%%|*}; envs=${spec#*|}
  env $envs timeout -k 10 300 python bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline --h2d-steps 0 ${BENCH_ARGS:-} > gpurun_out/abe_$n.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "$n failed rc=$rc"; tail -5 gpurun_out/abe_$n.log; exit $rc; fi
  grep "k_count stamps" gpurun_out/abe_$n.log | tail -1
  python - gpurun_out/abe_$n.log $n <<'PY'
import json, sys
j = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
st = {k: v for k, v in j["stages_ms_per_step"].items() if v > 0.05}
r = j.get("roofline") or {}
print(f'{sys.argv[2]:24s} {j["value"]/1e9:6.2f} G/s {j["ms_per_step"]:7.2f} ms {st} misses={r.get("lds_ops",{}).get("phase_b_records")}')
PY
done
