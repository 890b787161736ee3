export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --no-host --steps 20 --warmup 5"
tools/gpu_session.sh \
 "pytest_all::500::python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "benchA::300::python bench.py" \
 "benchB::120::$B --workload B" \
 "benchD::200::$B --workload D" \
 "profA::200::rocprofv3 --kernel-trace --stats -d gpurun_out/profA2 -o run --output-format csv -- $B --workload A"
