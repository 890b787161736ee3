#!/bin/bash
# Local helper: run tools/gpu_steps.sh <steps> on the gpurun box, after deleting this session's
# stale logs, then print the bench table (tools/abtab.py).  Output: gpurun_out/<name>.txt.
#   tools/gpurun_steps.sh <name> <timeout_s> <step> [<step> ...]
name=$1; tmo=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
cd "$ROOT"
GPU_STEPS_DRY=1 bash tools/gpu_steps.sh "$@" | while IFS= read -r spec; do
  t="${spec%%::*}"; rm -rf "gpurun_out/$t.log" "gpurun_out/prof_$t" gpurun_out/pmc_*_"$t" gpurun_out/pmc_*_"$t"_*.txt
done
q=""
for s in "$@"; do q="$q '$s'"; done
/usr/local/graft/bin/gpurun --timeout "$tmo" -- "bash tools/gpu_steps.sh$q" > "gpurun_out/$name.txt" 2>&1
rc=$?
grep -E "^\[gpurun\] (status|GPU-minutes)" "gpurun_out/$name.txt"
python3 tools/abtab.py "$@"
exit $rc
