#!/bin/bash
# Round-4 closing GPU call: the non-slow GPU suite, smoke, the default bench line, one bench line per k and the
# multi-k passes. Each GPU step has its own time limit; the chain stops at the first abnormal end.
set -o pipefail
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
O=gpurun_out/$TAG
timeout -k 10 700 python -u -m pytest tests -x -v -m "gpu and not slow" --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest exit $rc" >> $O/pytest_gpu.log
tail -3 $O/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { echo bench failed; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
for k in 21 33 55 63 77 99; do
  timeout -k 10 300 python bench.py --k $k --steps 5 --warmup 2 --no-cpu-baseline --h2d-steps 0 > $O/bench_k$k.json 2>&1 || { echo bench k=$k failed; tail -5 $O/bench_k$k.json; exit 1; }
done
timeout -k 10 300 python tools/bench_multik.py > $O/multik.log 2>&1 || { echo multik failed; tail -5 $O/multik.log; exit 1; }
tail -1 $O/multik.log | cut -c1-200
