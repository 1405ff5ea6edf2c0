set -o pipefail
timeout -k 10 600 python -u -m pytest tests -q -x -m "gpu and not slow" --timeout 300 --timeout-method thread > gpurun_out/pytest_fin2.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/pytest_fin2.log
