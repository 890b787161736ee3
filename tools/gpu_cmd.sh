set -o pipefail
mkdir -p gpurun_out/it16
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/it16/pytest.txt 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/it16/pytest.txt; exit 1; }
ALT=$GRAFT_REPO_ROOT/quic_amd/alt/libquic_fec_alt.so
for i in 1 2; do
timeout -k 10 120 python bench.py --workload B --no-cpu-baseline --no-host --steps 30 > gpurun_out/it16/Bnew$i.txt 2>&1 || exit 1
QFEC_LIB_PATH=$ALT timeout -k 10 120 python bench.py --workload B --no-cpu-baseline --no-host --steps 30 > gpurun_out/it16/Bold$i.txt 2>&1 || exit 1
done
