export TMPDIR=/tmp
tools/gpu_session.sh \
 "pytest_gpu::400::python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "B_ring::120::python bench.py --workload B --no-cpu-baseline --verify" \
 "B_ring_t4::120::QFEC_RING_TEAMS=4 python bench.py --workload B --no-cpu-baseline" \
 "B_ring_ns12::120::QFEC_RING_NS=12 python bench.py --workload B --no-cpu-baseline" \
 "B_ring_ns6t4::120::QFEC_RING_NS=6 QFEC_RING_TEAMS=4 python bench.py --workload B --no-cpu-baseline" \
 "B_ring_ns12t1::120::QFEC_RING_NS=12 QFEC_RING_TEAMS=1 python bench.py --workload B --no-cpu-baseline" \
 "D_ring::200::python bench.py --workload D --groups 16384 --steps 5 --warmup 2 --no-cpu-baseline --verify" \
 "D_ring_ns4::200::QFEC_RING_NS=4 python bench.py --workload D --groups 16384 --steps 5 --warmup 2 --no-cpu-baseline" \
 "D_ring_ns16::200::QFEC_RING_NS=16 python bench.py --workload D --groups 16384 --steps 5 --warmup 2 --no-cpu-baseline"
