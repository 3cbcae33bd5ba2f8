#!/bin/bash
# round 5: C3 TN stride / K-chunk phase probe
set -o pipefail
mkdir -p gpurun_out/r5j
timeout -k 10 200 tools/wide_lab tn128s > gpurun_out/r5j/lab_tn128s.txt 2>&1; rc=$?; cat gpurun_out/r5j/lab_tn128s.txt; exit $rc
