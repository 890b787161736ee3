export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --no-host --steps 10 --warmup 3 --workload D"
tools/gpu_session.sh \
 "dtests::400::python -u -m pytest tests/test_gpu_parity.py -k 'tile_many or syndrome_decode or config_d_full or options_parity or random_vs_oracle or golden' -x -q --timeout 120 --timeout-method thread" \
 "D_dcol::200::$B --verify" \
 "D_tile::200::$B --opt dcol=0" \
 "profD3::300::rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r03_D3 -o run --output-format csv -- $B"
