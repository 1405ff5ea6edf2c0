#!/bin/bash
# Round-3 GPU call: the default bench (rooflines of every main kernel), the multi-k read passes, and the slow
# full-size parity tests (C2 at k = 21, 63, 99 against the CPU restatement). Each GPU step has its own limit.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03r}
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -n 1 gpurun_out/bench_$TAG.log | cut -c1-200
timeout -k 10 400 python tools/bench_multik.py > gpurun_out/multik_$TAG.log 2>&1 || { echo multik failed; tail -5 gpurun_out/multik_$TAG.log; exit 1; }
tail -n 1 gpurun_out/multik_$TAG.log | cut -c1-300
[ -n "$NO_SLOW" ] && exit 0
timeout -k 10 900 python -u -m pytest tests -v -m "gpu and slow" -k "not c3_c4" --timeout 900 --timeout-method thread > gpurun_out/pytest_slow_$TAG.log 2>&1; rc=$?
echo "pytest exit $rc" >> gpurun_out/pytest_slow_$TAG.log
grep -E "passed|failed|PASSED|FAILED" gpurun_out/pytest_slow_$TAG.log | tail -8
[ $rc -ne 0 ] && exit 1
echo done
