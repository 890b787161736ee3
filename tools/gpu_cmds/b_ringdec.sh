B="python bench.py --no-cpu-baseline --no-host --steps 50 --warmup 5"
tools/gpu_session.sh \
 "tests::400::python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread" \
 "B_s1a::120::$B --workload B" \
 "B_s2a::120::$B --workload B --opt stream_static=2 --verify" \
 "B_s1b::120::$B --workload B" \
 "B_s2b::120::$B --workload B --opt stream_static=2" \
 "B_s2first::120::$B --workload B --opt stream_static=2 --parity first"
