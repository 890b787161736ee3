B="python bench.py --no-cpu-baseline --no-host --steps 20 --warmup 5"
tools/gpu_session.sh \
 "tests::400::python -u -m pytest tests/test_gpu_pp.py tests/test_gpu_parity.py -x -q -k 'pp or tile or 9008 or seal or open or known or stride' --timeout 120 --timeout-method thread" \
 "Da::200::$B --workload D" \
 "Db::200::$B --workload D" \
 "ppA::120::$B --workload A --pp" \
 "ppB::120::$B --workload B --pp"
