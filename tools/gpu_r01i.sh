export TMPDIR=/tmp
tools/gpu_session.sh \
 "pytest_gpu::400::python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "benchA::200::python bench.py --verify --no-cpu-baseline --no-host" \
 "benchB::200::python bench.py --workload B --verify --no-cpu-baseline --no-host" \
 "benchD::300::python bench.py --workload D --groups 16384 --steps 5 --warmup 2 --verify --no-cpu-baseline --no-host" \
 "profB::200::rocprofv3 --kernel-trace --stats -d gpurun_out/profB -o run --output-format csv -- python bench.py --workload B --no-cpu-baseline --no-host"
