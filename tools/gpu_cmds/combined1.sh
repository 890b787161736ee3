B="python bench.py --no-cpu-baseline --no-host --steps 20 --warmup 5"
tools/gpu_session.sh \
 "tests::400::python -u -m pytest tests/test_gpu_pp.py tests/test_gpu_timing.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread" \
 "ppA::120::$B --workload A --pp" \
 "ppB::120::$B --workload B --pp" \
 "benchD::200::$B --workload D --pp" \
 "benchD2::200::$B --workload D"
