export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --no-host --steps 10 --warmup 3"
tools/gpu_session.sh \
 "stests::400::python -u -m pytest tests/test_gpu_parity.py -k 'presets or any_small_block or options_parity or random_vs_oracle or golden or stream_ring or last_kernels or recovered or host_pointer or unsupported' -x -q --timeout 120 --timeout-method thread" \
 "A_graph::200::$B" \
 "A_nograph::200::$B --no-graph" \
 "profA::300::rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r03_A -o run --output-format csv -- $B" \
 "P_5_5::200::$B --preset 5,5" \
 "P_10_10::200::$B --preset 10,10" \
 "P_10_15::200::$B --preset 10,15" \
 "P_10_20::200::$B --preset 10,20" \
 "P_15_15::200::$B --preset 15,15" \
 "P_250_5::200::$B --preset 250,5" \
 "profP1010::300::rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r03_P1010 -o run --output-format csv -- $B --preset 10,10" \
 "D_def::200::$B --workload D --verify" \
 "D_c3::200::$B --workload D --opt dcol_cache=3" \
 "B_def::200::$B --workload B --verify" \
 "B_d3::200::$B --workload B --opt bsyn_depth=3" \
 "B_d4::200::$B --workload B --opt bsyn_depth=4" \
 "B_d6::200::$B --workload B --opt bsyn_depth=6" \
 "B_d7::200::$B --workload B --opt bsyn_depth=7"
