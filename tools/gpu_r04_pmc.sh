#!/bin/bash
# Round-4 PMC refresh at HEAD: for each config in CONFIGS ("tag:bench args" separated by ';'),
# one kernel-trace --stats run, then the PMC passes of tools/pmc_round.sh. Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
IFS=';' read -ra CFG <<< "$CONFIGS"
for c in "${CFG[@]}"; do
  tag=${c%%:*}; args=${c#*:}
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${tag}_ks -o run --output-format csv -- python3 $R/bench.py $args --no-cpu-baseline --h2d-steps 0 > $R/gpurun_out/${tag}_ks.log 2>&1) || { echo "stats $tag failed"; tail -5 gpurun_out/${tag}_ks.log; exit 1; }
  tail -1 gpurun_out/${tag}_ks.log | cut -c1-300
  TAG=$tag ARGS="$args --steps 1 --warmup 1 --no-cpu-baseline --no-profile-events --h2d-steps 0" bash tools/pmc_round.sh || exit 1
  python3 tools/pmc_summary.py $tag > gpurun_out/${tag}_summary.txt || exit 1
done
echo all done
