# same-box A/B on gf_stream cache policy: encode stores plain (st0), DMA loads default policy (ld0)
export TMPDIR=/tmp
B="python bench.py --workload B --no-cpu-baseline --no-host"
tools/gpu_session.sh \
 "s_base::200::QFEC_LIB_PATH=abtmp/lib_base.so $B" \
 "s_st0::200::QFEC_LIB_PATH=abtmp/lib_st0.so $B --verify" \
 "s_ld0::200::QFEC_LIB_PATH=abtmp/lib_ld0.so $B --verify" \
 "s_base2::200::QFEC_LIB_PATH=abtmp/lib_base.so $B" \
 "s_st02::200::QFEC_LIB_PATH=abtmp/lib_st0.so $B" \
 "s_ld02::200::QFEC_LIB_PATH=abtmp/lib_ld0.so $B"
