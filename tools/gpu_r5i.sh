#!/bin/bash
# round 5: LP = 128 TN with separate A / S rings (wproj3tn128_kernel) -- lab, C3 A/B, C3 pin test
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5i
timeout -k 10 120 tools/wide_lab tn128 > gpurun_out/r5i/lab_tn128.txt 2>&1 || { cat gpurun_out/r5i/lab_tn128.txt; exit 1; }
cat gpurun_out/r5i/lab_tn128.txt
CFGS="c3" STEPS=20 tools/ab_round.sh r5i "RSVD_TN128=0" "RSVD_TN128=1" "RSVD_TN128=2" "RSVD_TN128=1" || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bench_pin.py -k c3 > gpurun_out/r5i/pin.log 2>&1; rc=$?; tail -3 gpurun_out/r5i/pin.log; exit $rc
