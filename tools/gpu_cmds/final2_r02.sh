export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --no-host --steps 20 --warmup 5"
tools/gpu_session.sh \
 "tests::500::python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "benchD::300::python bench.py --workload D --verify --no-host --pp" \
 "profD::300::rocprofv3 --kernel-trace --stats -d gpurun_out/profD_f -o run --output-format csv -- $B --workload D" \
 "pmcD_F::200::rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_D_r02f/FETCH_SIZE -o run --output-format csv -- python bench.py --no-cpu-baseline --no-host --steps 3 --warmup 1 --workload D" \
 "pmcD_W::200::rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_D_r02f/WRITE_SIZE -o run --output-format csv -- python bench.py --no-cpu-baseline --no-host --steps 3 --warmup 1 --workload D" \
 "smoke::200::python -c 'import __graft_entry__ as g; g.smoke()'"
