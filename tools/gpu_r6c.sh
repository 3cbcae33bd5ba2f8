#!/bin/bash
# round 5: e4m3 NN on the v3-style wproj3nn8_kernel -- digests old / new, tests, bench A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6c
RSVD_NN8=0 timeout -k 10 120 python tools/digest_run.py > gpurun_out/r6c/digest0.txt 2>&1 || { cat gpurun_out/r6c/digest0.txt; exit 1; }
timeout -k 10 120 python tools/digest_run.py > gpurun_out/r6c/digest1.txt 2>&1 || { cat gpurun_out/r6c/digest1.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r6c/digest0.txt; grep -v amdgpu.ids gpurun_out/r6c/digest1.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bench_pin.py tests/test_gpu_wide.py > gpurun_out/r6c/tests.log 2>&1 || { tail -30 gpurun_out/r6c/tests.log; exit 1; }
tail -2 gpurun_out/r6c/tests.log
CFGS="c5" STEPS=10 tools/ab_round.sh r6c "" "RSVD_NN8=0" "" "RSVD_NN8=0"
