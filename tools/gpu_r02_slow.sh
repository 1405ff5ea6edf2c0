#!/bin/bash
# Round-2 GPU call: the slow (full-size) parity tests, then a rocprofv3 kernel-trace profile of the bench and
# single-GPU shares of C3 / C4. Each step has its own limit; an abnormal end stops the call.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r02s}
timeout -k 10 700 python -u -m pytest tests -v -m "gpu and slow" --timeout 900 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
echo "pytest exit $rc" >> gpurun_out/pytest_$TAG.log
grep -E "passed|failed|FAILED|ERROR" gpurun_out/pytest_$TAG.log | tail -15
if [ $rc -gt 1 ]; then echo "pytest ended abnormally ($rc)"; exit $rc; fi
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --h2d-steps 0 > $GRAFT_REPO_ROOT/gpurun_out/bench_prof_$TAG.log 2>&1 || { echo rocprof failed; tail -20 $GRAFT_REPO_ROOT/gpurun_out/bench_prof_$TAG.log; exit 1; }
tail -1 $GRAFT_REPO_ROOT/gpurun_out/bench_prof_$TAG.log
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --config C4 --reads-total 12500000 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c4share_$TAG.log 2>&1 || { echo c4 failed; tail -20 gpurun_out/bench_c4share_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_c4share_$TAG.log
timeout -k 10 300 python bench.py --config C3 --reads-total 12500000 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c3share_$TAG.log 2>&1 || { echo c3 failed; tail -20 gpurun_out/bench_c3share_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_c3share_$TAG.log
