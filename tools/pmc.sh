#!/bin/bash
# PMC passes over one bench workload, one counter group per rocprofv3 run (gfx950 slot
# limits: <= 8 SQ, <= 4 TCC (FETCH_SIZE takes 3, WRITE_SIZE 2)).  Output under
# gpurun_out/pmc_<W>_<tag>/<group>/.
#   tools/pmc.sh <workload A|B|D> <tag> [extra bench args]
W=${1:-A}; TAG=${2:-r01}; shift 2
export TMPDIR=/tmp
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH"; do
  name=$(echo $grp | cut -d' ' -f1)
  timeout -s KILL 90 rocprofv3 --pmc $grp -d gpurun_out/pmc_${W}_${TAG}/$name -o run --output-format csv -- python bench.py --workload $W --no-cpu-baseline --no-host --steps 5 --warmup 1 "$@" > gpurun_out/pmc_${W}_${TAG}_$name.txt 2>&1 || exit $?
done
