#!/bin/bash
# 2-rank host-transport rehearsal at the default pieces (16 for a host transport) and the multi-rank GPU tests
set -o pipefail
mkdir -p gpurun_out
A="--no-cpu-baseline --kmermap-sample-rows 0 --h2d-steps 0"
timeout -k 10 300 python bench.py --gpus 2 --transport host --steps 3 --warmup 1 $A > gpurun_out/mr_host2_def.log 2>&1 || { tail -5 gpurun_out/mr_host2_def.log; exit 1; }
tail -1 gpurun_out/mr_host2_def.log | python -c "import json,sys; j=json.loads(sys.stdin.read()); print('host2 default', j['value']/1e9, j['ms_per_step'], j['exchange']['ms_exposed_rank0'], j['exchange']['ms_transfers_rank0'])"
timeout -k 10 600 python -u -m pytest tests/test_multirank_gpu.py -x -q -m "gpu and not slow" --timeout 300 --timeout-method thread > gpurun_out/pytest_mr.log 2>&1 || { tail -20 gpurun_out/pytest_mr.log; exit 1; }
tail -1 gpurun_out/pytest_mr.log
