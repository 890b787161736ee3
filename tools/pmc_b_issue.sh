#!/bin/bash
# B issue/LDS probe: one counter group per rocprofv3 pass (<= 8 SQ, <= 2 GRBM).
export TMPDIR=/tmp
B="python bench.py --workload B --no-cpu-baseline --no-host --steps 5 --warmup 1"
i=0
for grp in "SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_VMEM SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_WAVES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $grp -d gpurun_out/pmc_Bissue/g$i -o run --output-format csv -- $B > gpurun_out/pmc_Bissue_g$i.txt 2>&1 || exit $?
done
