set -o pipefail
mkdir -p gpurun_out/it11
for W in A B; do for E in 0 1; do
QFEC_BENCH_NOEV=$E timeout -k 10 120 python bench.py --workload $W --no-cpu-baseline --no-host --steps 50 > gpurun_out/it11/${W}_noev$E.txt 2>&1 || exit 1
done; done
