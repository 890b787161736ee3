export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --no-host --steps 10 --warmup 3"
tools/gpu_session.sh \
 "tests::600::python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "P_5_5::200::$B --preset 5,5" \
 "P_10_10::200::$B --preset 10,10" \
 "P_10_15::200::$B --preset 10,15" \
 "P_10_20::200::$B --preset 10,20" \
 "P_15_15::200::$B --preset 15,15" \
 "P_250_5::200::$B --preset 250,5" \
 "profP1010::300::rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r03_P1010b -o run --output-format csv -- $B --preset 10,10" \
 "B_nt::200::$B --workload B" \
 "B_plain::200::$B --workload B --opt ring_nt=0" \
 "B_nt2::200::$B --workload B" \
 "B_plain2::200::$B --workload B --opt ring_nt=0"
