B="python bench.py --no-cpu-baseline --no-host --steps 20 --warmup 5"
tools/gpu_session.sh \
 "tests::400::python -u -m pytest tests/test_gpu_parity.py -x -q -k 'tile or 9008 or option' --timeout 120 --timeout-method thread" \
 "D1a::200::$B --workload D" \
 "D2a::200::$B --workload D --opt tile_pair=1 --verify" \
 "D1b::200::$B --workload D" \
 "D2b::200::$B --workload D --opt tile_pair=1"
