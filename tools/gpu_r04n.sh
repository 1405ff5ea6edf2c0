#!/bin/bash
# Round-4 closing GPU call at HEAD: tools/gpu_r04m.sh (suite, smoke, bench, per-k benches, multi-k), then the k = 99
# PMC passes. Stops at the first failure.
set -o pipefail
TAG=$TAG bash tools/gpu_r04m.sh || exit 1
CONFIGS="${TAG}_pmc_k99:--k 99" bash tools/gpu_r04_pmc.sh > gpurun_out/${TAG}_pmc99.log 2>&1 || { tail -5 gpurun_out/${TAG}_pmc99.log; exit 1; }
echo pmc done
