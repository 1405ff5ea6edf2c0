#!/bin/bash
# Round-2 GPU call: GPU tests (MARK selects: "gpu and not slow" by default), smoke, bench. Each GPU step has
# its own time limit; a crash, abort or time limit ends the call.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
MARK=${MARK:-"gpu and not slow"}
TAG=${TAG:-r02}
timeout -k 10 ${TEST_LIMIT:-700} python -u -m pytest tests -v -m "$MARK" --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
echo "pytest exit $rc" >> gpurun_out/pytest_$TAG.log
grep -E "passed|failed|FAILED|ERROR" gpurun_out/pytest_$TAG.log | tail -15
if [ $rc -gt 1 ]; then echo "pytest ended abnormally ($rc)"; exit $rc; fi
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo smoke failed; tail gpurun_out/smoke_$TAG.log; exit 1; }
cat gpurun_out/smoke_$TAG.log
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench_$TAG.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log
