#!/bin/bash
# GPU tests of the current tree (unless NO_TESTS), then A/B of library variants (tools/ab_env.sh arguments) at
# k = 21 (C2) and k = 63. Each GPU step has its own limit; an abnormal end stops the call.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-ab}
if [ -z "$NO_TESTS" ]; then
  TAG=$TAG NO_BENCH=1 bash tools/gpu_r02.sh || exit $?
fi
echo "== k=21"; bash tools/ab_env.sh "${@}" || exit $?
echo "== k=63"; BENCH_ARGS="--k 63" bash tools/ab_env.sh "${@}"
