set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_multirank_gpu.py -v -x --timeout 300 --timeout-method thread > gpurun_out/pytest_r03c.log 2>&1; rc=$?
echo "pytest exit $rc" >> gpurun_out/pytest_r03c.log
grep -E "passed|failed|FAILED|ERROR|Error" gpurun_out/pytest_r03c.log | tail -15
[ $rc -gt 1 ] && exit $rc
for own in hash minimizer; do
timeout -k 10 300 python bench.py --gpus 2 --transport host --k 63 --owner $own --steps 2 --warmup 1 --reads-per-gpu 2000000 --no-cpu-baseline --h2d-steps 0 --kmermap-sample-rows 0 > gpurun_out/bench_mr2_k63_${own}_r03c.log 2>&1 || { echo bench $own failed; tail -20 gpurun_out/bench_mr2_k63_${own}_r03c.log; exit 1; }
python -c "
import json,sys; j=json.loads(open('gpurun_out/bench_mr2_k63_${own}_r03c.log').read().strip().splitlines()[-1]); print('$own', j['value']/1e9, j['ms_per_step'], j['stages_ms_per_step'], j['exchange'])"
done
