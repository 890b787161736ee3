# round-1 close-out: tests, smoke, bench lines, rocprofv3 stats, PMC traffic for B
export TMPDIR=/tmp
tools/gpu_session.sh \
 "n_pytest_gpu::400::python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "n_smoke::120::python -c 'import __graft_entry__ as g; g.smoke()'" \
 "n_benchA::300::python bench.py --verify" \
 "n_benchB::300::python bench.py --workload B --verify --cpu-seconds 8" \
 "n_benchD::300::python bench.py --workload D --groups 16384 --steps 5 --warmup 2 --verify --cpu-groups 64 --cpu-seconds 8 --host-steps 1" \
 "n_profA::200::rocprofv3 --kernel-trace --stats -d gpurun_out/n_profA -o run --output-format csv -- python bench.py --no-cpu-baseline --no-host" \
 "n_profB::200::rocprofv3 --kernel-trace --stats -d gpurun_out/n_profB -o run --output-format csv -- python bench.py --workload B --no-cpu-baseline --no-host" \
 "n_profD::200::rocprofv3 --kernel-trace --stats -d gpurun_out/n_profD -o run --output-format csv -- python bench.py --workload D --groups 16384 --steps 5 --warmup 2 --no-cpu-baseline --no-host" \
 "n_pmcB::400::bash tools/pmc.sh B n"
