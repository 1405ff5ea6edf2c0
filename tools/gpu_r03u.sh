set -o pipefail
timeout -k 10 800 python -u -m pytest tests -q -m "gpu and not slow" --timeout 300 --timeout-method thread > gpurun_out/pytest_r03u.log 2>&1; rc=$?
tail -n 1 gpurun_out/pytest_r03u.log
[ $rc -ne 0 ] && { grep -E "^FAILED|Error" gpurun_out/pytest_r03u.log | head; exit 1; }
SKIP_PARITY=1 VARIANTS="cb2_7" PARITY_K="33 or 55 or 63 or wide or edge" KS="63 33" bash tools/gpu_ab3.sh
