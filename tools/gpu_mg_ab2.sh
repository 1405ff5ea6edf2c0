#!/bin/bash
# pair tests, then the paired bench for the tree and for exp/ variants given as arguments (name|ENV=V ...)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_fastq_pairs.py tests/test_fastq.py tests/test_fastq_file.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_pairs_mg.log 2>&1 || { tail -30 gpurun_out/pytest_pairs_mg.log; exit 1; }
tail -2 gpurun_out/pytest_pairs_mg.log
BENCH_ARGS="--input fastq-pairs" bash tools/ab_env.sh "new|X=1" "$@" "new2|X=1"
