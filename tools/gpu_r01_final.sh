export TMPDIR=/tmp
tools/gpu_session.sh \
 "pytest_gpu::400::python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "benchA::300::python bench.py --verify" \
 "benchB::300::python bench.py --workload B --verify --cpu-seconds 8" \
 "benchD::300::python bench.py --workload D --groups 16384 --steps 5 --warmup 2 --verify --cpu-groups 64 --cpu-seconds 8 --host-steps 1" \
 "dist2::300::QFEC_BENCH_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --verify" \
 "profA::200::rocprofv3 --kernel-trace --stats -d gpurun_out/profA -o run --output-format csv -- python bench.py --no-cpu-baseline --no-host" \
 "profB::200::rocprofv3 --kernel-trace --stats -d gpurun_out/profB -o run --output-format csv -- python bench.py --workload B --no-cpu-baseline --no-host" \
 "profD::200::rocprofv3 --kernel-trace --stats -d gpurun_out/profD -o run --output-format csv -- python bench.py --workload D --groups 16384 --steps 5 --warmup 2 --no-cpu-baseline --no-host" \
 "pmcA::400::bash tools/pmc.sh A r01" \
 "pmcB::400::bash tools/pmc.sh B r01" \
 "pmcD::400::bash tools/pmc.sh D r01 --groups 16384"
