export TMPDIR=/tmp
tools/gpu_session.sh \
 "pytest_gpu::400::python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "A_s2w4::120::python bench.py --workload A --no-cpu-baseline --verify" \
 "A_s3w3::120::QFEC_XOR_SLOTS=3 QFEC_XOR_WAVES=3 python bench.py --workload A --no-cpu-baseline --verify" \
 "A_s3w2::120::QFEC_XOR_SLOTS=3 QFEC_XOR_WAVES=2 python bench.py --workload A --no-cpu-baseline" \
 "A_s4w2::120::QFEC_XOR_SLOTS=4 QFEC_XOR_WAVES=2 python bench.py --workload A --no-cpu-baseline --verify" \
 "A_s2w3::120::QFEC_XOR_SLOTS=2 QFEC_XOR_WAVES=3 python bench.py --workload A --no-cpu-baseline" \
 "A_s4w1::120::QFEC_XOR_SLOTS=4 QFEC_XOR_WAVES=1 python bench.py --workload A --no-cpu-baseline"
