#!/bin/bash
# One GPU call's measurement round (run from the repo root on the GPU box): the default bench line, rocprofv3 kernel
# stats at k = 21 and k = 63, PMC passes at both (tools/pmc_round.sh; summaries via tools/pmc_summary.py), all under
# gpurun_out/ with the tag prefix $1 (e.g. r06b). Every step has its own time limit; the first failure ends the script.
set -o pipefail
P=${1:-r06}
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
step() { echo "[$(date +%T)] $*"; }
step bench
timeout -k 10 400 python3 -u bench.py > gpurun_out/${P}_bench.json 2> gpurun_out/${P}_bench.err || { echo "bench failed"; tail -5 gpurun_out/${P}_bench.err; exit 1; }
step kstats k21
bash tools/gpu_kstats.sh ${P}_kstats_k21 --steps 5 --warmup 2 --no-cpu-baseline --h2d-steps 0 --no-kmermap --no-k63 || exit 1
step kstats k63
bash tools/gpu_kstats.sh ${P}_kstats_k63 --k 63 --steps 5 --warmup 2 --no-cpu-baseline --h2d-steps 0 --no-kmermap || exit 1
step pmc k21
TAG=${P}_pmc_k21 ARGS="--steps 1 --warmup 1 --no-cpu-baseline --no-profile-events --h2d-steps 0 --no-kmermap --no-k63" bash tools/pmc_round.sh || exit 1
(cd $R && python3 tools/pmc_summary.py ${P}_pmc_k21 > /dev/null) || exit 1
step pmc k63
TAG=${P}_pmc_k63 ARGS="--k 63 --steps 1 --warmup 1 --no-cpu-baseline --no-profile-events --h2d-steps 0 --no-kmermap" bash tools/pmc_round.sh || exit 1
(cd $R && python3 tools/pmc_summary.py ${P}_pmc_k63 > /dev/null) || exit 1
# the raw per-pass CSVs stay on the box (the summaries carry every counter per kernel)
rm -rf gpurun_out/${P}_pmc_k21 gpurun_out/${P}_pmc_k63
step done
