#!/bin/bash
# Round-3 GPU call: GPU tests (not slow) on the tree with mixed three/four-word records, then an A/B of
# MHMKC_MIXED3=1/0 at k = 77 and 99 and the multi-k read passes. Each GPU step has its own limit.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03p}
if [ -z "$NO_TESTS" ]; then
timeout -k 10 800 python -u -m pytest tests -q -m "gpu and not slow" --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
echo "pytest exit $rc" >> gpurun_out/pytest_$TAG.log
grep -E "passed|failed" gpurun_out/pytest_$TAG.log | tail -3
if [ $rc -ne 0 ]; then echo "pytest failed ($rc)"; grep -E "^FAILED|Error" gpurun_out/pytest_$TAG.log | head -20; exit 1; fi
fi
for k in 77 99; do
  echo "== k=$k"; BENCH_ARGS="--k $k" bash tools/ab_env.sh "mx1|MHMKC_MIXED3=1" "mx0|MHMKC_MIXED3=0" || exit $?
done
timeout -k 10 400 python tools/bench_multik.py > gpurun_out/multik_$TAG.log 2>&1 || { echo multik failed; tail -5 gpurun_out/multik_$TAG.log; exit 1; }
tail -n 3 gpurun_out/multik_$TAG.log | cut -c1-600
echo done
