B="python bench.py --no-cpu-baseline --no-host --steps 20 --warmup 5"
tools/gpu_session.sh \
 "dtests::300::python -u -m pytest tests/test_gpu_parity.py -x -q -k 'tile or 9008' --timeout 120 --timeout-method thread" \
 "Da::200::$B --workload D" \
 "Db::200::$B --workload D" \
 "Dfirst::200::$B --workload D --parity first"
