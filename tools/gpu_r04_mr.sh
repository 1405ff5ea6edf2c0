#!/bin/bash
# Multi-rank bench rehearsals on the one-GPU box (ranks share the GPU): the exposed exchange at 2 ranks over the
# host transport with 4 and 16 pipelined pieces, then 8 ranks over the host transport and over RCCL's socket path.
set -o pipefail
mkdir -p gpurun_out
A="--no-cpu-baseline --kmermap-sample-rows 0 --h2d-steps 0"
timeout -k 10 300 python bench.py --gpus 2 --transport host --steps 3 --warmup 1 $A > gpurun_out/mr_host2_x4.log 2>&1 || { tail -5 gpurun_out/mr_host2_x4.log; exit 1; }
tail -1 gpurun_out/mr_host2_x4.log | python -c "import json,sys; j=json.loads(sys.stdin.read()); print('host2 x4', j['value']/1e9, j['ms_per_step'], j['exchange']['ms_exposed_rank0'], j['exchange']['ms_transfers_rank0'])"
MHMKC_XPIECES=16 timeout -k 10 300 python bench.py --gpus 2 --transport host --steps 3 --warmup 1 $A > gpurun_out/mr_host2_x16.log 2>&1 || { tail -5 gpurun_out/mr_host2_x16.log; exit 1; }
tail -1 gpurun_out/mr_host2_x16.log | python -c "import json,sys; j=json.loads(sys.stdin.read()); print('host2 x16', j['value']/1e9, j['ms_per_step'], j['exchange']['ms_exposed_rank0'], j['exchange']['ms_transfers_rank0'])"
timeout -k 10 600 python bench.py --gpus 8 --transport host --steps 3 --warmup 1 $A > gpurun_out/mr_host8.log 2>&1 || { tail -5 gpurun_out/mr_host8.log; exit 1; }
tail -1 gpurun_out/mr_host8.log | python -c "import json,sys; j=json.loads(sys.stdin.read()); print('host8', j['value']/1e9, j['ms_per_step'], j['exchange']['ms_exposed_rank0'], j['exchange']['ms_transfers_rank0'])"
timeout -k 10 600 python bench.py --gpus 8 --transport rccl-same-gpu --steps 2 --warmup 1 $A > gpurun_out/mr_rccl8.log 2>&1 || { tail -5 gpurun_out/mr_rccl8.log; exit 1; }
tail -1 gpurun_out/mr_rccl8.log | python -c "import json,sys; j=json.loads(sys.stdin.read()); print('rccl8', j['value']/1e9, j['ms_per_step'], j['exchange']['ms_exposed_rank0'], j['exchange']['ms_transfers_rank0'])"
