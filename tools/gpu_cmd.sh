set -o pipefail
mkdir -p gpurun_out/it17
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/it17/pytest.txt 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/it17/pytest.txt; exit 1; }
