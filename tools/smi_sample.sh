#!/bin/bash
# Sample the GPU's clocks, power and temperature every ~0.25 s into $1 until killed
# (diagnostics beside a bench run: tools/smi_sample.sh gpurun_out/smi.txt & ... kill $!).
out=${1:-gpurun_out/smi.txt}
while true; do
  echo "t=$(date +%s.%N)" >> "$out"
  timeout 5 rocm-smi --showclocks --showpower --showtemp >> "$out" 2>&1
  sleep 0.25
done
