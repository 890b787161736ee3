export TMPDIR=/tmp
tools/gpu_session.sh \
 "benchB::200::python bench.py --workload B --verify --no-cpu-baseline --no-host" \
 "benchD::300::python bench.py --workload D --groups 16384 --steps 5 --warmup 2 --verify --no-cpu-baseline --no-host" \
 "benchD_rc4::300::QFEC_ENC_RC=4 python bench.py --workload D --groups 16384 --steps 5 --warmup 2 --verify --no-cpu-baseline --no-host" \
 "benchD_rc2::300::QFEC_ENC_RC=2 python bench.py --workload D --groups 16384 --steps 5 --warmup 2 --verify --no-cpu-baseline --no-host" \
 "benchB_rc2::300::QFEC_ENC_RC=2 python bench.py --workload B --verify --no-cpu-baseline --no-host"
