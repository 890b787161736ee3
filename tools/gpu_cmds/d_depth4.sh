export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --no-host --steps 20 --warmup 5"
tools/gpu_session.sh \
 "dtests::300::python -u -m pytest tests/test_gpu_parity.py -x -q -k 'tile or 9008 or option' --timeout 120 --timeout-method thread" \
 "D6a::200::$B --workload D" \
 "D4a::200::$B --workload D --opt tile_depth=4" \
 "D6b::200::$B --workload D" \
 "D4b::200::$B --workload D --opt tile_depth=4" \
 "profD::300::rocprofv3 --kernel-trace --stats -d gpurun_out/profD3 -o run --output-format csv -- $B --workload D"
