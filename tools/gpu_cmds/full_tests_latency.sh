B="python bench.py --no-cpu-baseline --no-host --steps 10 --warmup 3"
tools/gpu_session.sh \
 "pytest_all::500::python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "latency::200::quic_amd/bin/dropin_latency --ref=oracle/_ref/libref_cauchy.so --iters=2000" \
 "D_first::200::$B --workload D --parity first" \
 "D_fixed_first::200::$B --workload D --parity first --loss-mode fixed" \
 "B_first::120::$B --workload B --parity first"
