#!/bin/bash
# Round-3 GPU call: rocprofv3 kernel stats of the C2 bench at k = 21, 63, 77, 99 (HEAD) and the k_count phase stamps
# (exp/libmhmkc_stamp.so, MHMKC_STAMP=1) at the same k.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
for k in 21 63 77 99; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_k${k}_r03j -o run --output-format csv -- python3 $R/bench.py --k $k --steps 5 --warmup 2 --no-cpu-baseline --h2d-steps 0 --kmermap-sample-rows 0 > $R/gpurun_out/bench_prof_k${k}_r03j.log 2>&1 || { echo "rocprof k=$k failed"; tail -20 $R/gpurun_out/bench_prof_k${k}_r03j.log; exit 1; }
  tail -1 $R/gpurun_out/bench_prof_k${k}_r03j.log | cut -c1-300
done
cd $R
for k in 21 63 77 99; do
  MHMKC_LIB=exp/libmhmkc_stamp.so timeout -k 10 300 python bench.py --k $k --steps 3 --warmup 1 --no-cpu-baseline --h2d-steps 0 --kmermap-sample-rows 0 > gpurun_out/bench_stamp_k${k}_r03j.log 2>&1 || { echo "stamp k=$k failed"; tail -20 gpurun_out/bench_stamp_k${k}_r03j.log; exit 1; }
  grep "stamps" gpurun_out/bench_stamp_k${k}_r03j.log | tail -1
done
echo done
