#!/bin/bash
# Round-3 GPU call: tools/gpu_r03l.sh (RCCL on one GPU, tests, smoke, bench), then the parity tests and an A/B at
# k = 21 / 63 of the library variants named in VARIANTS (exp/libmhmkc_<v>.so). Each GPU step has its own limit.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$SKIP_L" ]; then bash tools/gpu_r03l.sh || exit $?
elif [ -z "$SKIP_T" ]; then
  timeout -k 10 700 python -u -m pytest tests -q -m "gpu and not slow" --timeout 300 --timeout-method thread > gpurun_out/pytest_main.log 2>&1; rc=$?
  echo "main: $(tail -n 1 gpurun_out/pytest_main.log)"
  if [ $rc -ne 0 ]; then echo "main tests failed ($rc)"; grep -E "FAILED|Error" gpurun_out/pytest_main.log | head; exit 1; fi
fi
for v in $VARIANTS; do
  MHMKC_LIB=exp/libmhmkc_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -m "gpu and not slow" --timeout 300 --timeout-method thread > gpurun_out/pytest_parity_$v.log 2>&1; rc=$?
  echo "$v parity: $(tail -n 1 gpurun_out/pytest_parity_$v.log)"
  if [ $rc -ne 0 ]; then echo "variant $v parity failed ($rc)"; grep -E "FAILED|Error" gpurun_out/pytest_parity_$v.log | head; exit 1; fi
done
specs=("base|MHMKC_X=0")
for v in $VARIANTS; do specs+=("$v|MHMKC_LIB=exp/libmhmkc_$v.so"); done
echo "== k=21"; bash tools/ab_env.sh "${specs[@]}" || exit $?
echo "== k=63"; BENCH_ARGS="--k 63" bash tools/ab_env.sh "${specs[@]}" || exit $?
echo done
