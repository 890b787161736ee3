export TMPDIR=/tmp
tools/gpu_session.sh \
 "j_pytest_gpu::400::python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "j_smoke::120::python -c 'import __graft_entry__ as g; g.smoke()'" \
 "j_benchA::300::python bench.py --verify" \
 "j_benchB::300::python bench.py --workload B --verify --cpu-seconds 8" \
 "j_benchD::300::python bench.py --workload D --groups 16384 --steps 5 --warmup 2 --verify --cpu-groups 64 --cpu-seconds 8 --host-steps 1" \
 "j_profA::200::rocprofv3 --kernel-trace --stats -d gpurun_out/j_profA -o run --output-format csv -- python bench.py --no-cpu-baseline --no-host" \
 "j_profB::200::rocprofv3 --kernel-trace --stats -d gpurun_out/j_profB -o run --output-format csv -- python bench.py --workload B --no-cpu-baseline --no-host" \
 "j_profD::200::rocprofv3 --kernel-trace --stats -d gpurun_out/j_profD -o run --output-format csv -- python bench.py --workload D --groups 16384 --steps 5 --warmup 2 --no-cpu-baseline --no-host"
