export TMPDIR=/tmp
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH" "SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_IFETCH SQ_WAIT_INST_LDS"; do
  name=$(echo $grp | cut -d' ' -f1)
  timeout -s KILL 90 rocprofv3 --pmc $grp -d gpurun_out/pmcx/$name -o run --output-format csv -- python bench.py --workload B --no-cpu-baseline --no-host --steps 3 --warmup 1 > gpurun_out/pmcx_$name.txt 2>&1 || exit $?
done
