set -o pipefail
mkdir -p gpurun_out/it5
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "stream" > gpurun_out/it5/pytest.txt 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/it5/pytest.txt; exit 1; }
QFEC_STREAM_TIGHT=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "stream" > gpurun_out/it5/pytest_tight.txt 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/it5/pytest_tight.txt; exit 1; }
for T in 0 1; do for R in 6 7 8; do
QFEC_STREAM_TIGHT=$T QFEC_STREAM_ENC=1 QFEC_STREAM_RING=$R timeout -k 10 120 python bench.py --workload B --no-cpu-baseline --no-host --steps 20 --verify > gpurun_out/it5/B_t${T}_r$R.txt 2>&1 || exit 1
done; done
QFEC_STREAM_ENC=0 QFEC_STREAM_RING=8 timeout -k 10 120 python bench.py --workload B --no-cpu-baseline --no-host --steps 20 > gpurun_out/it5/B_flatenc.txt 2>&1
