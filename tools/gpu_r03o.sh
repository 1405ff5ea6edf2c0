#!/bin/bash
# Round-3 GPU call: bench + rocprof stats (tools/gpu_r03n.sh, NO_TESTS) then the PMC passes of tools/pmc_round.sh for
# C2 at k = 21 and 63 and the paired FASTQ path. Each GPU step has its own limit; an abnormal end stops the call.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
NO_TESTS=1 TAG=${TAG:-r03o} bash tools/gpu_r03n.sh || exit $?
[ -n "$NO_PMC" ] && exit 0
BASE="--steps 1 --warmup 1 --no-cpu-baseline --no-profile-events --h2d-steps 0 --kmermap-sample-rows 0"
TAG=r03_pmc_k21 ARGS="$BASE" bash tools/pmc_round.sh || exit 1
TAG=r03_pmc_k63 ARGS="$BASE --k 63" bash tools/pmc_round.sh || exit 1
TAG=r03_pmc_fqp ARGS="$BASE --input fastq-pairs" bash tools/pmc_round.sh || exit 1
echo done
