#!/bin/bash
# GPU tests, then A/B of the k_count table fit (MHMKC_CAP_LOAD) at k = 21 and 63, then k_count phase stamps.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r02j NO_BENCH=1 bash tools/gpu_r02.sh || exit $?
NO_TESTS=1 bash tools/gpu_ab2.sh "fit70|X=1" "nofit|MHMKC_CAP_LOAD=0" "fit60|MHMKC_CAP_LOAD=0.6" "fit80|MHMKC_CAP_LOAD=0.8" || exit $?
NO_PMC=1 bash tools/gpu_diag.sh
