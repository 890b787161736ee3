# gf_stream without the LDS mirror (R = 10 ring slots) vs base build (R = 8 + 2 KiB mirror)
export TMPDIR=/tmp
B="python bench.py --workload B --no-cpu-baseline --no-host"
tools/gpu_session.sh \
 "m_pytest::300::python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread" \
 "m_B_base::200::QFEC_LIB_PATH=abtmp/libquic_fec_base.so $B" \
 "m_B_new::200::$B --verify" \
 "m_B_base2::200::QFEC_LIB_PATH=abtmp/libquic_fec_base.so $B" \
 "m_B_new2::200::$B" \
 "m_B_r9::200::QFEC_STREAM_RING=9 $B" \
 "m_B_r8::200::QFEC_STREAM_RING=8 $B"
