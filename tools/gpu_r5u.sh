#!/bin/bash
# round 5: eig memset / memcpy launches, fused final conversions with U_w / V_w pieces -- bit-identity,
# wide / config / distributed tests, bench lines
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5u
timeout -k 10 120 python tools/digest_run.py > gpurun_out/r5u/digest.txt 2>&1 || { cat gpurun_out/r5u/digest.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r5u/digest.txt

timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_wide.py tests/test_gpu_configs.py tests/test_gpu_distributed.py tests/test_gpu_eig.py tests/test_gpu_bench_pin.py > gpurun_out/r5u/tests.log 2>&1 || { tail -30 gpurun_out/r5u/tests.log; exit 1; }
tail -2 gpurun_out/r5u/tests.log
CFGS="c5 c4 c3" STEPS=10 tools/ab_round.sh r5u ""
