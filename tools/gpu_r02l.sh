#!/bin/bash
# GPU tests, then A/B of the quad finalize (MHMKC_FINQ) at k = 21 and 63, then k_count phase stamps.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r02l NO_BENCH=1 bash tools/gpu_r02.sh || exit $?
NO_TESTS=1 bash tools/gpu_ab2.sh "finq|X=1" "nofinq|MHMKC_LIB=exp/libmhmkc_nofinq.so" "finq2|X=2" "nofinq2|MHMKC_LIB=exp/libmhmkc_nofinq.so" || exit $?
NO_PMC=1 bash tools/gpu_diag.sh
