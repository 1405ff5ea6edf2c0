#!/bin/bash
# Round-3 GPU call on HEAD: GPU tests (not slow), smoke, the default bench, and rocprofv3 --kernel-trace --stats of
# the C2 bench at the k in PROF_KS (default 21 63; "pairs" profiles the paired-FASTQ input at k = 21). MARK selects
# the tests (default: gpu and not slow). Each GPU step has its own time limit; an abnormal end stops the call.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03n}
R=$GRAFT_REPO_ROOT
if [ -z "$NO_TESTS" ]; then
timeout -k 10 ${TEST_LIMIT:-700} python -u -m pytest tests -v -m "${MARK:-gpu and not slow}" --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
echo "pytest exit $rc" >> gpurun_out/pytest_$TAG.log
grep -E "passed|failed" gpurun_out/pytest_$TAG.log | tail -3
if [ $rc -ne 0 ]; then echo "pytest failed ($rc)"; grep -E "FAILED|Error" gpurun_out/pytest_$TAG.log | head; exit 1; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo smoke failed; tail gpurun_out/smoke_$TAG.log; exit 1; }
cat gpurun_out/smoke_$TAG.log
fi
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -n 1 gpurun_out/bench_$TAG.log | cut -c1-300
cd /tmp
for k in ${PROF_KS:-21 63}; do
  args="--k $k"
  if [ "$k" = pairs ]; then args="--k 21 --input fastq-pairs"; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_k${k}_$TAG -o run --output-format csv -- python3 $R/bench.py $args --steps 5 --warmup 2 --no-cpu-baseline --h2d-steps 0 --kmermap-sample-rows 0 > $R/gpurun_out/bench_prof_k${k}_$TAG.log 2>&1 || { echo "rocprof $k failed"; tail -20 $R/gpurun_out/bench_prof_k${k}_$TAG.log; exit 1; }
  grep '^{' $R/gpurun_out/bench_prof_k${k}_$TAG.log | tail -n 1 | cut -c1-200
done
echo done
