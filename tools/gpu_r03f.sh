#!/bin/bash
# rocprofv3 kernel trace of the 2-rank host-transport bench at k = 63 with the supermer exchange (both ranks' kernels)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_smer_r03f -o run --output-format csv -- python3 $R/bench.py --gpus 2 --transport host --k 63 --owner minimizer --steps 2 --warmup 1 --reads-per-gpu 2000000 --no-cpu-baseline --h2d-steps 0 --kmermap-sample-rows 0 > $R/gpurun_out/bench_prof_smer_r03f.log 2>&1 || { echo rocprof failed; tail -20 $R/gpurun_out/bench_prof_smer_r03f.log; exit 1; }
tail -1 $R/gpurun_out/bench_prof_smer_r03f.log | cut -c1-300
find $R/gpurun_out/prof_smer_r03f -name "*kernel_stats.csv" | head
echo done
