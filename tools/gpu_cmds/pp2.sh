B="python bench.py --no-cpu-baseline --no-host --steps 10 --warmup 3"
tools/gpu_session.sh \
 "pp_tests::300::python -u -m pytest tests/test_gpu_pp.py -x -q --timeout 120 --timeout-method thread" \
 "ppA::120::$B --workload A --pp" \
 "ppB::120::$B --workload B --pp" \
 "ppD::200::$B --workload D --pp"
