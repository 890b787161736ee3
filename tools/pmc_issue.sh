#!/bin/bash
# Issue / wait / instruction-cache PMC passes over one bench workload (one rocprofv3 run per
# counter group, gfx950 slot limits).  Output under gpurun_out/pmci_<tag>/<group>/.
#   tools/pmc_issue.sh <tag> <bench args...>
TAG=$1; shift
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" \
           "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp -d gpurun_out/pmci_$TAG/g$i -o run --output-format csv -- python bench.py --no-cpu-baseline --no-host "$@" > gpurun_out/pmci_${TAG}_g$i.txt 2>&1 || exit $?
done
