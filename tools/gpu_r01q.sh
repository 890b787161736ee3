# D encode: two column words per lane (QFEC_W2=1, RC 4, PD 1) vs flat RC 8 / RC 4; parity first
export TMPDIR=/tmp
D="python bench.py --workload D --groups 16384 --steps 5 --warmup 2 --no-cpu-baseline --no-host"
tools/gpu_session.sh \
 "q_pytest_w2::300::QFEC_W2=1 QFEC_ENC_RC=4 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread" \
 "q_D_rc8::200::$D" \
 "q_D_w2::200::QFEC_W2=1 QFEC_ENC_RC=4 $D --verify" \
 "q_D_rc4::200::QFEC_ENC_RC=4 $D" \
 "q_D_w2b::200::QFEC_W2=1 QFEC_ENC_RC=4 $D" \
 "q_D_rc8b::200::$D"
