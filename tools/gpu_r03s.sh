#!/bin/bash
# Round-3 PMC passes (tools/pmc_round.sh) of the C2 bench at k = 77 and 99 (mixed three/four-word records).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
BASE="--steps 1 --warmup 1 --no-cpu-baseline --no-profile-events --h2d-steps 0 --kmermap-sample-rows 0"
TAG=r03_pmc_k77 ARGS="$BASE --k 77" bash tools/pmc_round.sh || exit 1
TAG=r03_pmc_k99 ARGS="$BASE --k 99" bash tools/pmc_round.sh || exit 1
echo done
