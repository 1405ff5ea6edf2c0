set -o pipefail
timeout -k 10 600 python -u -m pytest tests -q -x -m "gpu and not slow" --timeout 300 --timeout-method thread > gpurun_out/pytest_ex.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/pytest_ex.log
bash tools/ab_env.sh "new|X=1" "prev|MHMKC_LIB=exp/libmhmkc_0prev.so" "new2|X=1" "prev2|MHMKC_LIB=exp/libmhmkc_0prev.so" || exit 1
