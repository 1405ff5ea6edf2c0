#!/bin/bash
# Round-4 GPU call: focused tests (-k), then the whole non-slow GPU suite, smoke and one bench line.
# Each GPU step has its own time limit; the chain stops at the first abnormal end.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r04}
if [ -n "$FOCUS" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -v -s -m gpu -k "$FOCUS" --timeout 1150 --timeout-method thread > gpurun_out/pytest_focus_$TAG.log 2>&1; rc=$?
  echo "pytest exit $rc" >> gpurun_out/pytest_focus_$TAG.log
  tail -5 gpurun_out/pytest_focus_$TAG.log
  [ $rc -ne 0 ] && exit $rc
fi
if [ -z "$NOSUITE" ]; then
  timeout -k 10 700 python -u -m pytest tests -x -v -m "gpu and not slow" --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1; rc=$?
  echo "pytest exit $rc" >> gpurun_out/pytest_gpu_$TAG.log
  tail -5 gpurun_out/pytest_gpu_$TAG.log
  [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo smoke failed; tail gpurun_out/smoke_$TAG.log; exit 1; }
cat gpurun_out/smoke_$TAG.log
timeout -k 10 600 python bench.py $BENCH_ARGS > gpurun_out/bench_$TAG.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log
