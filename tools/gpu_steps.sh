#!/bin/bash
# One parameterised GPU session: every step this repo runs on the gpurun box, by name.
#   gpurun --timeout 1200 -- 'bash tools/gpu_steps.sh <step> [<step> ...]'
# Steps (output in gpurun_out/<label>.log; the session stops at the first fault, abort or
# time limit, see tools/gpu_session.sh):
#   tests                 the whole -m gpu suite
#   tests:<file|-k expr>  one test file (tests/test_gpu_pp.py) or a -k selection
#   testlib:<name>,<file> one test file against quic_amd/libquic_fec_<name>.so
#   mb:<name>             the microbenchmark binary tools/microbench/<name>
#   pg1:<W>[:<args>]      bench.py under torchrun with one rank and the RCCL process group kept
#                         (QFEC_BENCH_PG=1): the N > 1 control flow on one GPU
#   smoke                 __graft_entry__.smoke()
#   default               python bench.py (the driver's round-end line)
#   bench:<W>[:<args>]    bench.py --workload W --verify (W = A B C D), extra args after ':'
#   quick:<W>[:<args>]    bench.py --workload W, no CPU baseline, no host leg, 10 steps
#   preset:<k>,<m>        quick bench of a QuicR preset
#   prof:<W>[:<args>]     rocprofv3 --kernel-trace --stats of a quick bench
#   proflib:<name>,<W>[:<args>]  the same against quic_amd/libquic_fec_<name>.so
#   profp:<k>,<m>[:<args>] rocprofv3 --kernel-trace --stats of a QuicR preset's quick bench
#   abold:<W>[:<args>]    quick bench against quic_amd/libquic_fec_abold.so (an A/B build)
#   libq:<name>,<W>[:<args>]  quick bench against quic_amd/libquic_fec_<name>.so (W = A..D or
#                         P<k>_<m> for a QuicR preset)
#   aboldp:<k>,<m>        the same for a QuicR preset
#   pmc:<W>[:<args>]      tools/pmc.sh passes (FETCH/WRITE traffic, waves, issue mix)
#   pmcold:<W>[:<args>]   the same against quic_amd/libquic_fec_abold.so
#   pmclib:<name>,<W>[:<args>]  the same against quic_amd/libquic_fec_<name>.so
# Extra args use '+' for spaces: quick:B:--opt+bsyn_depth=3.  GPU_STEPS_DRY=1 prints the steps.
export TMPDIR=/tmp
specs=()
tags=()
for step in "$@"; do
  kind="${step%%:*}"; rest=""; [ "$step" != "$kind" ] && rest="${step#*:}"
  W="${rest%%:*}"; extra=""; [ "$rest" != "$W" ] && extra="${rest#*:}"
  extra="${extra//+/ }"
  tag=$(echo "$step" | tr -c 'A-Za-z0-9_\n' '_')
  # a repeated step gets its own log: <tag>_2, <tag>_3, ...
  n=1; base="$tag"; while [[ " ${tags[*]} " == *" $tag "* ]]; do n=$((n + 1)); tag="${base}_$n"; done
  tags+=("$tag")
  quick="python bench.py --no-cpu-baseline --no-host --steps 10 --warmup 3"
  case "$kind" in
    tests)
      if [ -z "$rest" ]; then sel="tests"
      elif [ -f "$rest" ]; then sel="$rest"
      else sel="tests -k '$rest'"; fi
      specs+=("$tag::900::python -u -m pytest $sel -m gpu -x -q --timeout 120 --timeout-method thread") ;;
    testlib) L="${W%%,*}"; F="${W#*,}"
            specs+=("$tag::900::QFEC_LIB_PATH=quic_amd/libquic_fec_$L.so python -u -m pytest $F -m gpu -x -q --timeout 120 --timeout-method thread") ;;
    mb)     specs+=("$tag::120::tools/microbench/$W") ;;
    pg1)    specs+=("$tag::300::QFEC_BENCH_PG=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --workload $W --no-host --steps 10 --warmup 3 $extra") ;;
    default) specs+=("default::600::python bench.py") ;;
    smoke)  specs+=("smoke::300::python -c 'import __graft_entry__ as g; g.smoke()'") ;;
    bench)  specs+=("$tag::600::python bench.py --workload $W --verify $extra") ;;
    quick)  specs+=("$tag::300::$quick --workload $W $extra") ;;
    preset) specs+=("$tag::300::$quick --preset $W $extra") ;;
    aboldp) specs+=("$tag::300::QFEC_LIB_PATH=quic_amd/libquic_fec_abold.so $quick --preset $W $extra") ;;
    libq)   L="${W%%,*}"; WW="${W#*,}"
            case "$WW" in P*_*) wl="--preset ${WW#P}"; wl="${wl/_/,}" ;; *) wl="--workload $WW" ;; esac
            specs+=("$tag::300::QFEC_LIB_PATH=quic_amd/libquic_fec_$L.so $quick $wl $extra") ;;
    abold)  specs+=("$tag::300::QFEC_LIB_PATH=quic_amd/libquic_fec_abold.so $quick --workload $W $extra") ;;
    prof)   specs+=("$tag::300::rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run --output-format csv -- $quick --workload $W $extra") ;;
    proflib) L="${W%%,*}"; WW="${W#*,}"
            case "$WW" in P*_*) wl="--preset ${WW#P}"; wl="${wl/_/,}" ;; *) wl="--workload $WW" ;; esac
            specs+=("$tag::300::QFEC_LIB_PATH=quic_amd/libquic_fec_$L.so rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run --output-format csv -- $quick $wl $extra") ;;
    profp)  specs+=("$tag::300::rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run --output-format csv -- $quick --preset $W $extra") ;;
    pmc)    specs+=("$tag::600::bash tools/pmc.sh $W $tag $extra") ;;
    pmclib) L="${W%%,*}"; WW="${W#*,}"
            specs+=("$tag::600::QFEC_LIB_PATH=quic_amd/libquic_fec_$L.so bash tools/pmc.sh $WW $tag $extra") ;;
    pmcold) specs+=("$tag::600::QFEC_LIB_PATH=quic_amd/libquic_fec_abold.so bash tools/pmc.sh $W $tag $extra") ;;
    *) echo "unknown step: $step"; exit 2 ;;
  esac
done
if [ -n "$GPU_STEPS_DRY" ]; then printf '%s\n' "${specs[@]}"; exit 0; fi
exec tools/gpu_session.sh "${specs[@]}"
