#!/bin/bash
# Round-3 PMC call on HEAD: the counter passes of tools/pmc_round.sh for C2 k = 21, k = 63 and the paired FASTQ path
# (k_fq_merge*), then rocprofv3 kernel-trace stats of the C2 and k = 63 benches. Each GPU step has its own limit.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
BASE="--steps 1 --warmup 1 --no-cpu-baseline --no-profile-events --h2d-steps 0 --kmermap-sample-rows 0"
TAG=r03_pmc_k21 ARGS="$BASE" bash tools/pmc_round.sh || exit 1
TAG=r03_pmc_k63 ARGS="$BASE --k 63" bash tools/pmc_round.sh || exit 1
TAG=r03_pmc_fqp ARGS="$BASE --input fastq-pairs" bash tools/pmc_round.sh || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r03b -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --h2d-steps 0 --kmermap-sample-rows 0 > $R/gpurun_out/bench_prof_r03b.log 2>&1 || { echo rocprof failed; tail -20 $R/gpurun_out/bench_prof_r03b.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_k63_r03b -o run --output-format csv -- python3 $R/bench.py --k 63 --steps 5 --warmup 2 --no-cpu-baseline --h2d-steps 0 --kmermap-sample-rows 0 > $R/gpurun_out/bench_prof_k63_r03b.log 2>&1 || { echo rocprof k63 failed; tail -20 $R/gpurun_out/bench_prof_k63_r03b.log; exit 1; }
echo done
