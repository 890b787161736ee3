# same-box A/B: coarse vmcnt ladder below 16 in gf_stream (coarse) vs exact 16-way tree (base)
export TMPDIR=/tmp
B="python bench.py --workload B --no-cpu-baseline --no-host"
tools/gpu_session.sh \
 "p_B_base::200::QFEC_LIB_PATH=abtmp/lib_base.so $B" \
 "p_B_coarse::200::QFEC_LIB_PATH=abtmp/lib_coarse.so $B --verify" \
 "p_B_base2::200::QFEC_LIB_PATH=abtmp/lib_base.so $B" \
 "p_B_coarse2::200::QFEC_LIB_PATH=abtmp/lib_coarse.so $B" \
 "p_B_base3::200::QFEC_LIB_PATH=abtmp/lib_base.so $B" \
 "p_B_coarse3::200::QFEC_LIB_PATH=abtmp/lib_coarse.so $B"
