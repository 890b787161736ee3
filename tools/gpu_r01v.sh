# D encode with one 16-output chunk (QFEC_ENC_RC=16: no W/Z re-expansion, 2 waves/SIMD) vs RC 8
export TMPDIR=/tmp
D="python bench.py --workload D --groups 16384 --steps 5 --warmup 2 --no-cpu-baseline --no-host"
tools/gpu_session.sh \
 "v_pytest16::300::QFEC_ENC_RC=16 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread" \
 "v_D_rc8::200::$D" \
 "v_D_rc16::200::QFEC_ENC_RC=16 $D --verify" \
 "v_D_rc8b::200::$D" \
 "v_D_rc16b::200::QFEC_ENC_RC=16 $D"
