export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --no-host --steps 10 --warmup 3 --pp"
tools/gpu_session.sh \
 "pptests::300::python -u -m pytest tests/test_gpu_pp.py -m gpu -x -q --timeout 120 --timeout-method thread" \
 "A_pp0::200::$B --workload A" \
 "A_pp1::200::$B --workload A --opt pp_hash=1" \
 "B_pp0::200::$B --workload B" \
 "B_pp1::200::$B --workload B --opt pp_hash=1" \
 "profA_pp::300::rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r03_App -o run --output-format csv -- $B --workload A"
