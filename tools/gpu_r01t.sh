# same-box A/B: gf_stream decode stores nt (dnt) vs plain (base); slots layout as well
export TMPDIR=/tmp
B="python bench.py --workload B --no-cpu-baseline --no-host"
tools/gpu_session.sh \
 "t_base::200::QFEC_LIB_PATH=abtmp/lib_base.so $B" \
 "t_dnt::200::QFEC_LIB_PATH=abtmp/lib_dnt.so $B --verify" \
 "t_base2::200::QFEC_LIB_PATH=abtmp/lib_base.so $B" \
 "t_dnt2::200::QFEC_LIB_PATH=abtmp/lib_dnt.so $B" \
 "t_base_sl::200::QFEC_LIB_PATH=abtmp/lib_base.so $B --decode-layout slots" \
 "t_dnt_sl::200::QFEC_LIB_PATH=abtmp/lib_dnt.so $B --decode-layout slots --verify"
