set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_dbjg.py tests/test_cpp_adapter.py -q -x -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_dbjg.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/pytest_dbjg.log
bash tools/ab_env.sh "base|X=1" "stamp|MHMKC_LIB=exp/libmhmkc_stamp.so MHMKC_PRINT_STAMPS=1" "cb4|MHMKC_LIB=exp/libmhmkc_cb4.so" "probe32|MHMKC_LIB=exp/libmhmkc_probe32.so" || exit 1
