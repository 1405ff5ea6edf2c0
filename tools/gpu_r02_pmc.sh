#!/bin/bash
# Round-2 PMC passes (tools/pmc_round.sh: one rocprofv3 --pmc run per counter group, kernel trace only) for C2 at
# k = 21, at k = 63 and from FASTQ text. Summaries are made on the host afterwards (tools/pmc_summary.py).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
BASE="--steps 1 --warmup 1 --no-cpu-baseline --no-profile-events --h2d-steps 0 --kmermap-sample-rows 0"
TAG=pmcf_k21 ARGS="$BASE" bash tools/pmc_round.sh || exit $?
TAG=pmcf_k63 ARGS="$BASE --k 63" bash tools/pmc_round.sh || exit $?
TAG=pmcf_fq ARGS="$BASE --input fastq" bash tools/pmc_round.sh || exit $?
echo pmc done
