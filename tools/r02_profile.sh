export TMPDIR=/tmp
P="python bench.py --no-cpu-baseline --no-host --steps 10 --warmup 3"
tools/gpu_session.sh \
 "pytest::400::python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "profA::200::rocprofv3 --kernel-trace --stats -d gpurun_out/profA -o run --output-format csv -- $P --workload A" \
 "profB::200::rocprofv3 --kernel-trace --stats -d gpurun_out/profB -o run --output-format csv -- $P --workload B" \
 "profD::300::rocprofv3 --kernel-trace --stats -d gpurun_out/profD -o run --output-format csv -- $P --workload D" \
 "pmcB_F::120::rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcB_F -o run --output-format csv -- python bench.py --no-cpu-baseline --no-host --steps 3 --warmup 1 --workload B" \
 "pmcB_W::120::rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcB_W -o run --output-format csv -- python bench.py --no-cpu-baseline --no-host --steps 3 --warmup 1 --workload B" \
 "pmcD_F::300::rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcD_F -o run --output-format csv -- python bench.py --no-cpu-baseline --no-host --steps 3 --warmup 1 --workload D" \
 "pmcD_W::300::rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcD_W -o run --output-format csv -- python bench.py --no-cpu-baseline --no-host --steps 3 --warmup 1 --workload D" \
 "pmcA_F::120::rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcA_F -o run --output-format csv -- python bench.py --no-cpu-baseline --no-host --steps 3 --warmup 1 --workload A" \
 "pmcA_W::120::rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcA_W -o run --output-format csv -- python bench.py --no-cpu-baseline --no-host --steps 3 --warmup 1 --workload A"
