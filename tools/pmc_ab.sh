#!/bin/bash
# One --pmc pass (SQ instruction mix) per library variant, on the C2 bench: rocprofv3 kernel-trace only.
#   bash tools/pmc_ab.sh name=path ...   (path "" = the in-tree library)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmcab
rm -rf $OUT
CNT=${CNT:-"SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS"}
cd /tmp
for spec in "$@"; do
  n=${spec%%=*}; lib=${spec#*=}
  if [ -n "$lib" ]; then export MHMKC_LIB=$GRAFT_REPO_ROOT/$lib; else unset MHMKC_LIB; fi
  timeout -s KILL 240 rocprofv3 --pmc $CNT --kernel-trace -d $OUT/$n -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-profile-events --h2d-steps 0 ${BENCH_ARGS:-} > $OUT.$n.log 2>&1 || { echo "pass $n failed"; tail -5 $OUT.$n.log; exit 1; }
  echo "$n done"
done
