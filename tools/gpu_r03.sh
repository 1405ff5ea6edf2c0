#!/bin/bash
# Round-3 GPU call: GPU tests (MARK / PYTEST_ARGS select), smoke, the default bench, and the multi-rank launcher
# rehearsal (2 ranks over the host transport on this one GPU; --gpus 8 over RCCL must fail cleanly here). Each
# GPU step has its own time limit; a crash, abort or time limit ends the call.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
MARK=${MARK:-"gpu and not slow"}
TAG=${TAG:-r03}
if [ -z "$NO_TESTS" ]; then
timeout -k 10 ${TEST_LIMIT:-700} python -u -m pytest tests -v -m "$MARK" --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
echo "pytest exit $rc" >> gpurun_out/pytest_$TAG.log
grep -E "passed|failed|FAILED|ERROR" gpurun_out/pytest_$TAG.log | tail -15
if [ $rc -gt 1 ]; then echo "pytest ended abnormally ($rc)"; exit $rc; fi
fi
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo smoke failed; tail gpurun_out/smoke_$TAG.log; exit 1; }
cat gpurun_out/smoke_$TAG.log
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench_$TAG.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log
[ -n "$NO_MR" ] && exit 0
timeout -k 10 400 python bench.py --gpus 2 --transport host --steps 3 --warmup 1 --reads-per-gpu ${MR_READS:-2000000} --no-cpu-baseline --h2d-steps 0 --kmermap-sample-rows 0 > gpurun_out/bench_mr2_$TAG.log 2>&1 || { echo bench mr2 failed; tail -20 gpurun_out/bench_mr2_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_mr2_$TAG.log
timeout -k 10 120 python bench.py --gpus 8 --steps 1 --warmup 0 --reads-per-gpu 10000 --no-cpu-baseline --h2d-steps 0 > gpurun_out/bench_g8_$TAG.log 2>&1; rc=$?
echo "--gpus 8 on one GPU: exit $rc (expected non-zero)"; tail -3 gpurun_out/bench_g8_$TAG.log
[ $rc -ne 0 ] && [ $rc -ne 124 ] && [ $rc -ne 137 ] || { echo "unexpected --gpus 8 result $rc"; exit 1; }
echo done
