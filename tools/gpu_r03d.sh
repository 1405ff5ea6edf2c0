#!/bin/bash
# Round-3 GPU call: GPU tests (incl. the supermer exchange and shared-counter tests), then an A/B of the
# unconditional k_count prefetch (new default) against the old conditional one (exp/libmhmkc_pf0.so) at k = 21 and
# 63, then 2-rank host-transport benches at k = 63 with records (hash owner) and supermers (minimizer owner).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03d}
timeout -k 10 900 python -u -m pytest tests -v -m "gpu and not slow" --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
echo "pytest exit $rc" >> gpurun_out/pytest_$TAG.log
grep -E "passed|failed|FAILED|ERROR" gpurun_out/pytest_$TAG.log | tail -25
if [ $rc -gt 1 ]; then echo "pytest ended abnormally ($rc)"; exit $rc; fi
STEPS=5 bash tools/ab_env.sh "new21|X=1" "old21|MHMKC_LIB=exp/libmhmkc_pf0.so" "new21b|X=1" || exit 1
STEPS=5 BENCH_ARGS="--k 63" bash tools/ab_env.sh "new63|X=1" "old63|MHMKC_LIB=exp/libmhmkc_pf0.so" || exit 1
for own in hash minimizer; do
timeout -k 10 300 python bench.py --gpus 2 --transport host --k 63 --owner $own --steps 2 --warmup 1 --reads-per-gpu 2000000 --no-cpu-baseline --h2d-steps 0 --kmermap-sample-rows 0 > gpurun_out/bench_mr2_k63_${own}_$TAG.log 2>&1 || { echo bench $own failed; tail -20 gpurun_out/bench_mr2_k63_${own}_$TAG.log; exit 1; }
python -c "
import json,sys; j=json.loads(open('gpurun_out/bench_mr2_k63_${own}_$TAG.log').read().strip().splitlines()[-1]); print('$own', round(j['value']/1e9,2), j['ms_per_step'], j['stages_ms_per_step'], j['exchange'])"
done
echo done
