export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --no-host --steps 20 --warmup 5"
tools/gpu_session.sh \
 "tests::500::python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "smoke::200::python -c 'import __graft_entry__ as g; g.smoke()'" \
 "benchD::300::python bench.py --workload D --verify --no-host" \
 "profD::300::rocprofv3 --kernel-trace --stats -d gpurun_out/profD_f2 -o run --output-format csv -- $B --workload D" \
 "benchA::300::python bench.py --verify"
