#!/bin/bash
# Round-3 GPU call: A/B of the batched-claim phase A (exp/libmhmkc_fasta.so vs exp/libmhmkc_base.so) at k = 21,
# the k_count parity tests on the rebuilt in-tree library, then the slow C3/C4 rank-share tests (progress printed).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=10 bash tools/ab_env.sh "base|MHMKC_LIB=exp/libmhmkc_base.so" "fasta|MHMKC_LIB=exp/libmhmkc_fasta.so" \
  "base2|MHMKC_LIB=exp/libmhmkc_base.so" "fasta2|MHMKC_LIB=exp/libmhmkc_fasta.so" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_parity_r03h.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_parity_r03h.log
if [ $rc -ne 0 ]; then echo "parity failed ($rc)"; exit $rc; fi
timeout -k 10 1000 python -u -m pytest tests/test_multirank_gpu.py -k c3_c4 -v -s -x -m gpu --timeout 900 --timeout-method thread > gpurun_out/pytest_share_r03h.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error|rank|parent" gpurun_out/pytest_share_r03h.log | tail -30
exit $rc
