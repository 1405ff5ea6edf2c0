#!/bin/bash
# rocprofv3 kernel-trace stats of one bench configuration: TAG, then bench arguments
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
tag=$1; shift
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$tag -o run --output-format csv -- python3 $R/bench.py "$@" > $R/gpurun_out/$tag.log 2>&1) || { echo "stats $tag failed"; tail -5 gpurun_out/$tag.log; exit 1; }
python3 tools/kstats.py gpurun_out/$tag
