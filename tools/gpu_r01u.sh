# spread of the default bench line on one box: 3 x default A, 1 x A with 200 steps
export TMPDIR=/tmp
A="python bench.py --no-cpu-baseline --no-host"
tools/gpu_session.sh \
 "u_A1::200::$A" "u_A2::200::$A" "u_A3::200::$A" \
 "u_A200::300::$A --steps 200 --warmup 20"
