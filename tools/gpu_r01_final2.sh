export TMPDIR=/tmp
tools/gpu_session.sh \
 "f2_pytest_gpu::400::python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "f2_benchA::300::python bench.py --verify" \
 "f2_benchB::300::python bench.py --workload B --verify --cpu-seconds 8" \
 "f2_benchD::300::python bench.py --workload D --groups 16384 --steps 5 --warmup 2 --verify --cpu-groups 64 --cpu-seconds 8 --host-steps 1" \
 "f2_profA::200::rocprofv3 --kernel-trace --stats -d gpurun_out/f2_profA -o run --output-format csv -- python bench.py --no-cpu-baseline --no-host" \
 "f2_profB::200::rocprofv3 --kernel-trace --stats -d gpurun_out/f2_profB -o run --output-format csv -- python bench.py --workload B --no-cpu-baseline --no-host" \
 "f2_profD::200::rocprofv3 --kernel-trace --stats -d gpurun_out/f2_profD -o run --output-format csv -- python bench.py --workload D --groups 16384 --steps 5 --warmup 2 --no-cpu-baseline --no-host" \
 "f2_pmcB::400::bash tools/pmc.sh B f2" \
 "f2_pmcD::400::bash tools/pmc.sh D f2 --groups 16384"
