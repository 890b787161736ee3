set -o pipefail
mkdir -p gpurun_out/it12
for W in A B; do
timeout -k 10 120 python bench.py --workload $W --no-cpu-baseline --no-host --steps 50 --verify > gpurun_out/it12/${W}.txt 2>&1 || exit 1
done
QFEC_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --no-cpu-baseline --no-host --verify > gpurun_out/it12/dist2.txt 2>&1
