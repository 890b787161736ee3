export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --no-host --steps 20 --warmup 5"
tools/gpu_session.sh \
 "benchA::300::python bench.py --verify" \
 "benchB::300::python bench.py --workload B --verify --no-host" \
 "benchC::300::$B --workload C --verify" \
 "benchD::300::python bench.py --workload D --verify --no-host" \
 "profA::200::rocprofv3 --kernel-trace --stats -d gpurun_out/profA_f -o run --output-format csv -- $B --workload A" \
 "profB::200::rocprofv3 --kernel-trace --stats -d gpurun_out/profB_f -o run --output-format csv -- $B --workload B" \
 "gloo2C::300::QFEC_BENCH_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 --verify"
