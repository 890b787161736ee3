export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --no-host --steps 10 --warmup 3"
tools/gpu_session.sh \
 "stests::400::python -u -m pytest tests/test_gpu_parity.py -k 'presets or any_small_block or tile_many or syndrome_decode or options_parity or random_vs_oracle or golden or stream_ring or last_kernels' -x -q --timeout 120 --timeout-method thread" \
 "D_c0::200::$B --workload D --opt dcol_cache=0" \
 "D_c1::200::$B --workload D --opt dcol_cache=1" \
 "D_c2::200::$B --workload D --opt dcol_cache=2" \
 "P_5_5::200::$B --preset 5,5" \
 "P_10_10::200::$B --preset 10,10" \
 "P_10_15::200::$B --preset 10,15" \
 "P_10_20::200::$B --preset 10,20" \
 "P_15_15::200::$B --preset 15,15" \
 "P_250_5::200::$B --preset 250,5"
