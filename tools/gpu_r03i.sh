#!/bin/bash
# Round-3 GPU call: the multi-rank tests on the pipelined record exchange (default on), then host-transport 2-rank
# benches with the pipeline on / off at k = 21 and k = 63 (hash owner: records on the wire).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03i}
timeout -k 10 900 python -u -m pytest tests/test_multirank_gpu.py -v -s -x -m gpu --timeout 600 --timeout-method thread > gpurun_out/pytest_mr_$TAG.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_mr_$TAG.log | tail -8
if [ $rc -ne 0 ]; then echo "pytest failed ($rc)"; exit $rc; fi
for k in 21 63; do
  for xp in 1 0; do
    MHMKC_XPIPE=$xp timeout -k 10 300 python bench.py --gpus 2 --transport host --k $k --steps 5 --warmup 2 --no-cpu-baseline --h2d-steps 0 --kmermap-sample-rows 0 > gpurun_out/bench_x${xp}_k${k}_$TAG.log 2>&1 || { echo "bench k=$k xpipe=$xp failed"; tail -20 gpurun_out/bench_x${xp}_k${k}_$TAG.log; exit 1; }
    python - gpurun_out/bench_x${xp}_k${k}_$TAG.log <<'PY'
import json, sys
j = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], round(j["value"] / 1e9, 2), "G/s", j["ms_per_step"], "ms", json.dumps(j["exchange"]))
PY
  done
done
echo done
