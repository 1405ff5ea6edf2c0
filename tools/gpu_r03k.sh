#!/bin/bash
# Round-3 PMC call on HEAD: the counter passes of tools/pmc_round.sh for C2 at k = 21, 63, 77 and
# the paired FASTQ path (k_fq_merge*), then the k_count phase stamps (exp/libmhmkc_stamp.so) at k = 21, 63, 77, 99.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
BASE="--steps 1 --warmup 1 --no-cpu-baseline --no-profile-events --h2d-steps 0 --kmermap-sample-rows 0"
TAG=r03_pmc_k21 ARGS="$BASE" bash tools/pmc_round.sh || exit 1
TAG=r03_pmc_k63 ARGS="$BASE --k 63" bash tools/pmc_round.sh || exit 1
TAG=r03_pmc_k77 ARGS="$BASE --k 77" bash tools/pmc_round.sh || exit 1
TAG=r03_pmc_fqp ARGS="$BASE --input fastq-pairs" bash tools/pmc_round.sh || exit 1
for k in 21 63 77 99; do
  MHMKC_PRINT_STAMPS=1 MHMKC_LIB=exp/libmhmkc_stamp.so timeout -k 10 300 python bench.py --k $k --steps 3 --warmup 1 --no-cpu-baseline --h2d-steps 0 --kmermap-sample-rows 0 > gpurun_out/bench_stamp_k${k}_r03k.log 2>&1 || { echo "stamp k=$k failed"; tail -20 gpurun_out/bench_stamp_k${k}_r03k.log; exit 1; }
  echo "k=$k $(grep 'k_count stamps' gpurun_out/bench_stamp_k${k}_r03k.log | tail -1)"
done
echo done
