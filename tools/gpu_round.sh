#!/bin/bash
# One GPU call: tests, smoke, bench, rocprofv3 kernel-trace stats. Each GPU step has its own time limit
# and the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r05}
MARK=${MARK:-"gpu and not slow"}
timeout -k 10 ${TEST_LIMIT:-900} python -u -m pytest tests -x -v -m "$MARK" --timeout 170 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1; rc=$?
echo "pytest exit $rc" >> gpurun_out/pytest_gpu_$TAG.log
tail -5 gpurun_out/pytest_gpu_$TAG.log
# test failures (1) still allow the measurements; a crash, abort or time limit ends the call
if [ $rc -gt 1 ]; then echo "pytest ended abnormally ($rc)"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo smoke failed; tail gpurun_out/smoke_$TAG.log; exit 1; }
cat gpurun_out/smoke_$TAG.log
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log
[ -n "$NO_PROF" ] && exit 0
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --h2d-steps 0 --no-kmermap > $GRAFT_REPO_ROOT/gpurun_out/bench_prof_$TAG.log 2>&1 || { echo rocprof failed; tail -20 $GRAFT_REPO_ROOT/gpurun_out/bench_prof_$TAG.log; exit 1; }
tail -1 $GRAFT_REPO_ROOT/gpurun_out/bench_prof_$TAG.log
find $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -name "*stats*" | head
