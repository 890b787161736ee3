# same-box A/B: coefficient prefetch ring in gf_apply (new) vs base build
export TMPDIR=/tmp
D="python bench.py --workload D --groups 16384 --steps 5 --warmup 2 --no-cpu-baseline --no-host"
tools/gpu_session.sh \
 "l_D_base::200::QFEC_LIB_PATH=abtmp/libquic_fec_base.so $D" \
 "l_D_new::200::$D" \
 "l_D_base2::200::QFEC_LIB_PATH=abtmp/libquic_fec_base.so $D" \
 "l_D_new2::200::$D"
