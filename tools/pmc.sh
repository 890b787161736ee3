#!/bin/bash
# PMC passes over one bench workload, one counter group per rocprofv3 run (gfx950 slot
# limits: <= 8 SQ, <= 4 TCC (FETCH_SIZE takes 3, WRITE_SIZE 2)).  Output under
# gpurun_out/pmc_<W>_<tag>/<group>/ (per-dispatch rows in run_counter_collection.csv).
#   tools/pmc.sh <workload A|B|D|P<k>_<m>> <tag> [extra bench args]
# PMC_SETS (optional): counter groups separated by ';' instead of the default five.
W=${1:-A}; TAG=${2:-r01}; shift 2
export TMPDIR=/tmp
DEFAULT_SETS="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE;SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU;SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH"
IFS=';' read -r -a sets <<< "${PMC_SETS:-$DEFAULT_SETS}"
case "$W" in
  P*_*) km="${W#P}"; wl="--preset ${km/_/,}"; wn="$W" ;;   # P10_20: the QuicR preset (10, 20)
  *)    wl="--workload $W"; wn="$W" ;;
esac
for grp in "${sets[@]}"; do
  name=$(echo $grp | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d gpurun_out/pmc_${wn}_${TAG}/$name -o run --output-format csv -- python bench.py $wl --no-cpu-baseline --no-host --steps 5 --warmup 1 "$@" > gpurun_out/pmc_${wn}_${TAG}_$name.txt 2>&1 || exit $?
done
