#!/bin/bash
# round 5: LP = 512 Gram from pre-split pieces (lab, bit-identity against gram_split4)
set -o pipefail
mkdir -p gpurun_out/r5q
timeout -k 10 120 tools/wide_lab gpieces > gpurun_out/r5q/gpieces.txt 2>&1; rc=$?; cat gpurun_out/r5q/gpieces.txt; exit $rc
