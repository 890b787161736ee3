export TMPDIR=/tmp
tools/gpu_session.sh \
 "pytest_gpu::300::python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread" \
 "benchA::240::python bench.py --workload A --verify" \
 "benchB::240::python bench.py --workload B --verify --cpu-seconds 8" \
 "benchD::300::python bench.py --workload D --groups 16384 --steps 5 --warmup 2 --verify --cpu-groups 64 --cpu-seconds 8" \
 "profA::240::rocprofv3 --kernel-trace --stats -d gpurun_out/profA -o run --output-format csv -- python bench.py --workload A --no-cpu-baseline" \
 "profB::240::rocprofv3 --kernel-trace --stats -d gpurun_out/profB -o run --output-format csv -- python bench.py --workload B --no-cpu-baseline"
