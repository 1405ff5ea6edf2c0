#!/bin/bash
# k_fq_merge / k_fq_merge_pack work: the pair tests, then a paired-FASTQ bench A/B (HEAD build vs the tree)
# and one stamped run (MHMKC_MGSTAMP build) for the merge phase split.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_fastq_pairs.py tests/test_fastq.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_pairs_mg.log 2>&1 || { tail -30 gpurun_out/pytest_pairs_mg.log; exit 1; }
tail -2 gpurun_out/pytest_pairs_mg.log
BENCH_ARGS="--input fastq-pairs" bash tools/ab_env.sh "prev|MHMKC_LIB=exp/libmhmkc_0prev.so" "new|X=1" "prev2|MHMKC_LIB=exp/libmhmkc_0prev.so" "new2|X=1" || exit 1
if [ -n "$STAMP" ]; then
  BENCH_ARGS="--input fastq-pairs" bash tools/ab_env.sh "mgst|MHMKC_LIB=exp/libmhmkc_mgstamp.so MHMKC_PRINT_STAMPS=1" || exit 1
  grep "k_fq_merge stamps" gpurun_out/abe_mgst.log | tail -1
fi
