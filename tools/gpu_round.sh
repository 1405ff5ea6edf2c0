#!/bin/bash
# One GPU call: tests, smoke, bench, rocprofv3 kernel-trace stats. Each GPU step has its own time limit
# and the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01}
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest exit $rc" >> gpurun_out/pytest_gpu.log
tail -5 gpurun_out/pytest_gpu.log
# test failures (1) still allow the measurements; a crash, abort or time limit ends the call
if [ $rc -gt 1 ]; then echo "pytest ended abnormally ($rc)"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/bench_prof.log 2>&1 || { echo rocprof failed; tail -20 $GRAFT_REPO_ROOT/gpurun_out/bench_prof.log; exit 1; }
tail -1 $GRAFT_REPO_ROOT/gpurun_out/bench_prof.log
find $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -name "*stats*" | head
