#!/bin/bash
# round 5: LP = 128 TN rings + K phases -- lab identity, wide / pin tests, C3 A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5k
timeout -k 10 120 tools/wide_lab tn128 > gpurun_out/r5k/lab_tn128.txt 2>&1 || { cat gpurun_out/r5k/lab_tn128.txt; exit 1; }
cat gpurun_out/r5k/lab_tn128.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_wide.py tests/test_gpu_bench_pin.py -k "not workload" > gpurun_out/r5k/tests.log 2>&1 || { tail -30 gpurun_out/r5k/tests.log; exit 1; }
tail -2 gpurun_out/r5k/tests.log
CFGS="c3" STEPS=20 tools/ab_round.sh r5k "RSVD_TN128=0" "RSVD_TN128=1" "RSVD_TN128=0" "RSVD_TN128=1"
