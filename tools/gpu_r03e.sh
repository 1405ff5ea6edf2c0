#!/bin/bash
# Round-3 GPU call: the multi-rank GPU tests, then 2-rank host-transport benches at k = 63 (records vs supermers).
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r03e}
timeout -k 10 600 python -u -m pytest tests/test_multirank_gpu.py tests/test_minimizer_gpu.py -v -x --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
echo "pytest exit $rc" >> gpurun_out/pytest_$TAG.log
grep -E "passed|failed|FAILED|ERROR" gpurun_out/pytest_$TAG.log | tail -25
if [ $rc -ne 0 ]; then echo "pytest failed ($rc)"; exit $rc; fi
for own in hash minimizer; do
timeout -k 10 300 python bench.py --gpus 2 --transport host --k 63 --owner $own --steps 2 --warmup 1 --reads-per-gpu 2000000 --no-cpu-baseline --h2d-steps 0 --kmermap-sample-rows 0 > gpurun_out/bench_mr2_k63_${own}_$TAG.log 2>&1 || { echo bench $own failed; tail -20 gpurun_out/bench_mr2_k63_${own}_$TAG.log; exit 1; }
python -c "
import json,sys; j=json.loads(open('gpurun_out/bench_mr2_k63_${own}_$TAG.log').read().strip().splitlines()[-1]); print('$own', round(j['value']/1e9,2), j['ms_per_step'], j['stages_ms_per_step'], j['exchange'])"
done
echo done
