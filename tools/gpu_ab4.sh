#!/bin/bash
# GPU parity tests of the main library, then an A/B of environment switches (ENVS: "name|ENV=V ...") and library
# variants (VARIANTS, exp/libmhmkc_<v>.so) at the k values in KS (TESTFILE: the parity tests run first; BENCH_ARGS:
# extra bench.py arguments). Each GPU step has its own limit.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest ${TESTFILE:-tests/test_gpu_parity.py} -x -q -m "gpu and not slow" --timeout 300 --timeout-method thread > gpurun_out/pytest_parity_main.log 2>&1; rc=$?
echo "main parity: $(tail -n 1 gpurun_out/pytest_parity_main.log)"
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/pytest_parity_main.log | head; exit 1; fi
for v in $VARIANTS; do
  MHMKC_LIB=exp/libmhmkc_$v.so timeout -k 10 400 python -u -m pytest ${TESTFILE:-tests/test_gpu_parity.py} -x -q -m "gpu and not slow" -k "${PARITY_K:-not nothing}" --timeout 300 --timeout-method thread > gpurun_out/pytest_parity_$v.log 2>&1; rc=$?
  echo "$v parity: $(tail -n 1 gpurun_out/pytest_parity_$v.log)"
  if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/pytest_parity_$v.log | head; exit 1; fi
done
specs=("base|MHMKC_X=0")
for e in $ENVS; do specs+=("$e"); done
for v in $VARIANTS; do specs+=("$v|MHMKC_LIB=exp/libmhmkc_$v.so"); done
for k in ${KS:-21 63}; do
  echo "== k=$k"; BENCH_ARGS="--k $k ${BENCH_ARGS:-}" bash tools/ab_env.sh "${specs[@]}" || exit $?
done
echo done
