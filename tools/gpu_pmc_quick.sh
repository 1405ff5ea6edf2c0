#!/bin/bash
# A few SQ counter passes (instruction mix, waits) over one bench configuration: TAG, then bench arguments
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
tag=$1; shift
rm -rf $R/gpurun_out/$tag
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  (cd /tmp && timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace -d $R/gpurun_out/$tag/p$i -o run --output-format csv -- python3 $R/bench.py "$@" > $R/gpurun_out/$tag.p$i.log 2>&1) || { echo "pass $i failed"; tail -5 $R/gpurun_out/$tag.p$i.log; exit 1; }
done
python3 tools/pmc_summary.py $tag > gpurun_out/${tag}_summary.txt && grep -A16 "k_fq_merge\b\|k_fq_merge<\|k_fq_merge_pack" gpurun_out/${tag}_summary.txt | head -60
