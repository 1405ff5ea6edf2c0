#!/bin/bash
# GPU tests, then A/B of the per-wave miss queues (MHMKC_WAVEQ) at k = 21 and 63, then k_count phase stamps.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r02k NO_BENCH=1 bash tools/gpu_r02.sh || exit $?
NO_TESTS=1 bash tools/gpu_ab2.sh "waveq|MHMKC_CAP_LOAD=0" "noq|MHMKC_CAP_LOAD=0 MHMKC_LIB=exp/libmhmkc_noq.so" "waveq2|MHMKC_CAP_LOAD=0" || exit $?
NO_PMC=1 bash tools/gpu_diag.sh
