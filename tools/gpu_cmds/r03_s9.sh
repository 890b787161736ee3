export TMPDIR=/tmp
tools/gpu_session.sh \
 "pptests::300::python -u -m pytest tests/test_gpu_pp.py -m gpu -x -q --timeout 120 --timeout-method thread" \
 "benchA::400::python bench.py --verify --pp" \
 "benchB::400::python bench.py --workload B --verify --pp --host-groups 65536" \
 "benchC::400::python bench.py --workload C --verify --no-host" \
 "benchD::600::python bench.py --workload D --verify --host-groups 16384 --steps 10 --warmup 3" \
 "profA::300::rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r03_Afinal -o run --output-format csv -- python bench.py --no-cpu-baseline --no-host" \
 "profB::300::rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r03_Bfinal -o run --output-format csv -- python bench.py --workload B --no-cpu-baseline --no-host" \
 "profD::300::rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r03_Dfinal -o run --output-format csv -- python bench.py --workload D --no-cpu-baseline --no-host --steps 5 --warmup 2"
