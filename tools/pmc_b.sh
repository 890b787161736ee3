#!/bin/bash
# PMC passes over bench workload $1 (env passed through), one counter group per pass.
W=${1:-B}; TAG=${2:-stage}
export TMPDIR=/tmp
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU" "FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU"; do
  name=$(echo $grp | cut -d' ' -f1)
  timeout -k 10 200 rocprofv3 --pmc $grp -d gpurun_out/pmc_${W}_${TAG}/$name -o run --output-format csv -- python bench.py --workload $W --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/pmc_${W}_${TAG}_$name.log 2>&1 || exit $?
done
