#!/bin/bash
# Run tools/wide_lab modes on the GPU box under a time limit: tools/lab_run.sh mode [mode ...]
set -o pipefail
mkdir -p gpurun_out
for m in "$@"; do
  timeout -k 10 240 ./tools/wide_lab $m > gpurun_out/lab_$m.txt 2>&1 || { cat gpurun_out/lab_$m.txt; exit 1; }
  cat gpurun_out/lab_$m.txt
done
