export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --no-host --steps 10 --warmup 3 --workload D"
tools/gpu_session.sh \
 "valu::120::tools/microbench/valu_rate" \
 "newtests::300::python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_parity.py -k 'config_d_full or shards_gloo' -x -v --timeout 200 --timeout-method thread" \
 "benchA2::200::python bench.py --no-cpu-baseline --no-host" \
 "D_base::200::$B" \
 "D_occ2_p5::200::$B --opt tile_occ2=1 --opt tile_depth=5" \
 "D_occ2_6::200::$B --opt tile_occ2=1 --opt tile_depth=6 --opt tile_pair=0" \
 "D_occ2_4::200::$B --opt tile_occ2=1 --opt tile_depth=4 --opt tile_pair=0"
