#!/bin/bash
# Round-3 GPU call: multi-rank tests (with the slow C3 / C4 rank-share tests), then the supermer kernel profile.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03g}
R=$GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest tests/test_multirank_gpu.py -v -x -m gpu --timeout 1500 --timeout-method thread --durations=10 > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
echo "pytest exit $rc" >> gpurun_out/pytest_$TAG.log
grep -E "passed|failed|FAILED|ERROR|s call" gpurun_out/pytest_$TAG.log | tail -25
if [ $rc -ne 0 ]; then echo "pytest failed ($rc)"; exit $rc; fi
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_smer_$TAG -o run --output-format csv -- python3 $R/bench.py --gpus 2 --transport host --k 63 --owner minimizer --steps 2 --warmup 1 --reads-per-gpu 2000000 --no-cpu-baseline --h2d-steps 0 --kmermap-sample-rows 0 > $R/gpurun_out/bench_prof_smer_$TAG.log 2>&1 || { echo rocprof failed; tail -20 $R/gpurun_out/bench_prof_smer_$TAG.log; exit 1; }
tail -1 $R/gpurun_out/bench_prof_smer_$TAG.log | cut -c1-400
echo done
