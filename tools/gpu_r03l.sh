#!/bin/bash
# Round-3 GPU call: libmhmkc's RCCL exchange with the ranks on one GPU (per-rank NCCL_HOSTID, socket transport), then
# the GPU tests, smoke, the default bench and a 2-rank bench over that RCCL path. Each GPU step has its own limit.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03l}
timeout -k 10 600 python -u -m pytest tests/test_multirank_gpu.py -v -k rccl --timeout 300 --timeout-method thread > gpurun_out/pytest_rccl_$TAG.log 2>&1; rc=$?
echo "pytest exit $rc" >> gpurun_out/pytest_rccl_$TAG.log
grep -E "passed|failed|FAILED|ERROR" gpurun_out/pytest_rccl_$TAG.log | tail -15
if [ $rc -gt 1 ]; then echo "rccl pytest ended abnormally ($rc)"; exit $rc; fi
timeout -k 10 300 python bench.py --gpus 2 --transport rccl-same-gpu --steps 3 --warmup 1 --reads-per-gpu 2000000 --no-cpu-baseline --h2d-steps 0 --kmermap-sample-rows 0 > gpurun_out/bench_mr2_rccl_$TAG.log 2>&1 || { echo bench rccl mr2 failed; tail -30 gpurun_out/bench_mr2_rccl_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_mr2_rccl_$TAG.log | cut -c1-600
[ -n "$ONLY_RCCL" ] && exit 0
timeout -k 10 700 python -u -m pytest tests -v -m "gpu and not slow" -k "not rccl" --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
echo "pytest exit $rc" >> gpurun_out/pytest_$TAG.log
grep -E "passed|failed|FAILED|ERROR" gpurun_out/pytest_$TAG.log | tail -15
if [ $rc -gt 1 ]; then echo "pytest ended abnormally ($rc)"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo smoke failed; tail gpurun_out/smoke_$TAG.log; exit 1; }
cat gpurun_out/smoke_$TAG.log
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log | cut -c1-400
echo done
