# D encode code-size probe: FLAT RC = 8 (78 KB of code), 4 (40 KB), 2 (20 KB); I-cache PMC
export TMPDIR=/tmp
D="python bench.py --workload D --groups 16384 --steps 5 --warmup 2 --no-cpu-baseline --no-host"
tools/gpu_session.sh \
 "k_D_rc8::200::$D" \
 "k_D_rc4::200::QFEC_ENC_RC=4 $D" \
 "k_D_rc2::200::QFEC_ENC_RC=2 $D" \
 "k_B_rc8::200::QFEC_STREAM_ENC=0 python bench.py --workload B --no-cpu-baseline --no-host" \
 "k_pmc_ic::90::timeout -s KILL 60 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE -d gpurun_out/k_pmc_ic -o run --output-format csv -- $D"
