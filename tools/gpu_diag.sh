#!/bin/bash
# Diagnostics call: k_count phase stamps (MHMKC_STAMP build) at k = 21 and 63, then the PMC passes of the FASTQ
# ingest path (tools/pmc_round.sh). Each GPU step has its own limit; an abnormal end stops the call.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for k in 21 63; do
  MHMKC_PRINT_STAMPS=1 MHMKC_LIB=exp/libmhmkc_stamp.so timeout -k 10 300 python bench.py --k $k --steps 3 --warmup 1 --no-cpu-baseline --h2d-steps 0 --kmermap-sample-rows 0 > gpurun_out/stamp_k$k.log 2>&1 || { echo "stamp k=$k failed"; tail -5 gpurun_out/stamp_k$k.log; exit 1; }
  grep "k_count stamps" gpurun_out/stamp_k$k.log | tail -1
done
[ -n "$NO_PMC" ] && exit 0
TAG=pmc_fq ARGS="--input fastq --steps 1 --warmup 1 --no-cpu-baseline --no-profile-events --h2d-steps 0 --kmermap-sample-rows 0" bash tools/pmc_round.sh
