set -o pipefail
mkdir -p gpurun_out/it14
for i in 1 2 3; do
timeout -k 10 120 python bench.py --workload A --no-cpu-baseline --no-host --steps 50 > gpurun_out/it14/new$i.txt 2>&1 || exit 1
QFEC_LIB_PATH=$GRAFT_REPO_ROOT/quic_amd/alt/libquic_fec_alt.so timeout -k 10 120 python bench.py --workload A --no-cpu-baseline --no-host --steps 50 > gpurun_out/it14/old$i.txt 2>&1 || exit 1
done
