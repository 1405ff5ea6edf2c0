#!/bin/bash
# PMC passes (each counter group in its own rocprofv3 run, kernel-trace only; no sys/runtime trace).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-pmc}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
rm -rf $OUT
ARGS=${ARGS:-"--steps 1 --warmup 1 --no-cpu-baseline --no-profile-events --h2d-steps 0 --no-kmermap"}
cd /tmp
i=0
GROUPS_DEFAULT=(
 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
 "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
 "SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA"
 "TA_BUSY_avr TA_BUSY_max TD_TD_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum"
 "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"
)
for grp in "${GROUPS_DEFAULT[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace -d $OUT/p$i -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS > $OUT.p$i.log 2>&1 || { echo "pass $i failed: $grp"; tail -5 $OUT.p$i.log; exit 1; }
done
echo done
