set -o pipefail
mkdir -p gpurun_out/it9
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/it9/pytest.txt 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/it9/pytest.txt; exit 1; }
timeout -k 10 120 python bench.py --workload B --no-cpu-baseline --no-host --steps 20 --verify > gpurun_out/it9/B.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/it9/prof -o run --output-format csv -- python bench.py --workload B --no-cpu-baseline --no-host --steps 10 > gpurun_out/it9/B_prof.txt 2>&1
