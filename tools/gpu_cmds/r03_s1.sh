export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --no-host --steps 20 --warmup 5"
tools/gpu_session.sh \
 "tests::700::python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "smoke::200::python -c 'import __graft_entry__ as g; g.smoke()'" \
 "benchA::200::$B --verify" \
 "benchB::200::$B --workload B --verify" \
 "benchD::300::$B --workload D --verify" \
 "profBD::400::rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r03a -o run --output-format csv -- $B --workload B" \
 "profD::400::rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r03a_D -o run --output-format csv -- $B --workload D --steps 5"
