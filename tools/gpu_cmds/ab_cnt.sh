B="python bench.py --no-cpu-baseline --no-host --steps 50 --warmup 5"
BASE="QFEC_LIB_PATH=quic_amd/libquic_fec_base.so"
tools/gpu_session.sh \
 "tests::500::python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "A_new1::120::$B --workload A" \
 "A_base1::120::$BASE $B --workload A" \
 "A_new2::120::$B --workload A" \
 "A_base2::120::$BASE $B --workload A" \
 "B_new1::120::$B --workload B" \
 "B_base1::120::$BASE $B --workload B" \
 "B_new2::120::$B --workload B" \
 "B_base2::120::$BASE $B --workload B"
