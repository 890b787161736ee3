#!/bin/bash
# Run a sequence of GPU steps on the gpurun box; stop at the first fault/abort/timeout.
# Usage: tools/gpu_session.sh "<name>::<timeout_s>::<command>" ...
# Each step's output goes to gpurun_out/<name>.log.  Exit codes 0 and 1 (test
# failures) continue; anything else (124/137 timeout, 134 abort, 139 segfault, ...)
# ends the session.
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for spec in "$@"; do
  name="${spec%%::*}"; rest="${spec#*::}"
  tmo="${rest%%::*}"; cmd="${rest#*::}"
  echo "=== [$name] (timeout ${tmo}s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$tmo" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc in $(( $(date +%s) - start ))s"
  tail -n 15 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "=== stopping: step $name exited $rc"
    exit $rc
  fi
done
exit 0
