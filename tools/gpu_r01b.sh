export TMPDIR=/tmp
tools/gpu_session.sh \
 "pytest_gpu::400::python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread" \
 "B_stage::120::python bench.py --workload B --no-cpu-baseline" \
 "B_apply_pd2::120::QFEC_NO_STAGE=1 python bench.py --workload B --no-cpu-baseline" \
 "B_apply_pd1::120::QFEC_NO_STAGE=1 QFEC_PD=1 python bench.py --workload B --no-cpu-baseline" \
 "B_apply_pd3::120::QFEC_NO_STAGE=1 QFEC_PD=3 python bench.py --workload B --no-cpu-baseline" \
 "D_apply::200::QFEC_NO_STAGE=1 python bench.py --workload D --groups 16384 --steps 5 --warmup 2 --no-cpu-baseline" \
 "A_nodma::120::QFEC_NO_DMA=1 python bench.py --workload A --no-cpu-baseline"
