#!/bin/bash
# Round-2 measurement call: GPU tests (fast, then slow full-size), smoke, the default bench (C2, with the CPU
# baseline, H2D-inclusive leg and KmerMap timing), the k = 63 bench, and rocprofv3 kernel-trace stats of both.
# Each GPU step has its own limit; an abnormal end stops the call.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r02f}
R=$GRAFT_REPO_ROOT
if [ -z "$SKIP_TESTS" ]; then
TAG=$TAG NO_BENCH=1 bash tools/gpu_r02.sh || exit $?
timeout -k 10 700 python -u -m pytest tests -v -m "gpu and slow" --timeout 900 --timeout-method thread > gpurun_out/pytest_slow_$TAG.log 2>&1; rc=$?
echo "pytest exit $rc" >> gpurun_out/pytest_slow_$TAG.log
grep -E "passed|failed|FAILED|ERROR" gpurun_out/pytest_slow_$TAG.log | tail -5
if [ $rc -ne 0 ]; then echo "slow pytest failed ($rc)"; exit 1; fi
fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo smoke failed; tail gpurun_out/smoke_$TAG.log; exit 1; }
cat gpurun_out/smoke_$TAG.log | grep smoke
timeout -k 10 500 python bench.py > gpurun_out/bench_$TAG.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log
timeout -k 10 400 python bench.py --k 63 --no-cpu-baseline > gpurun_out/bench_k63_$TAG.log 2>&1 || { echo bench k63 failed; tail -20 gpurun_out/bench_k63_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_k63_$TAG.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --h2d-steps 0 --kmermap-sample-rows 0 > $R/gpurun_out/bench_prof_$TAG.log 2>&1 || { echo rocprof failed; tail -20 $R/gpurun_out/bench_prof_$TAG.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_k63_$TAG -o run --output-format csv -- python3 $R/bench.py --k 63 --steps 5 --warmup 2 --no-cpu-baseline --h2d-steps 0 --kmermap-sample-rows 0 > $R/gpurun_out/bench_prof_k63_$TAG.log 2>&1 || { echo rocprof k63 failed; tail -20 $R/gpurun_out/bench_prof_k63_$TAG.log; exit 1; }
echo done
