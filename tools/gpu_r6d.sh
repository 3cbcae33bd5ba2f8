#!/bin/bash
# round 5: bf16 NN at LP = 128 on wproj3_kernel -- digests old / new, tests, bench A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6d
RSVD_NN3_128=0 timeout -k 10 120 python tools/digest_run.py > gpurun_out/r6d/digest0.txt 2>&1 || { cat gpurun_out/r6d/digest0.txt; exit 1; }
timeout -k 10 120 python tools/digest_run.py > gpurun_out/r6d/digest1.txt 2>&1 || { cat gpurun_out/r6d/digest1.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r6d/digest0.txt; grep -v amdgpu.ids gpurun_out/r6d/digest1.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_wide.py tests/test_gpu_configs.py > gpurun_out/r6d/tests.log 2>&1 || { tail -30 gpurun_out/r6d/tests.log; exit 1; }
tail -2 gpurun_out/r6d/tests.log
CFGS="c3 c2" STEPS=10 tools/ab_round.sh r6d "" "RSVD_NN3_128=0" "" "RSVD_NN3_128=0"
