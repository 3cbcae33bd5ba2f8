#!/bin/bash
# round 5: tridiagonalisation skips dead row slots -- bit-identity, eig / wide tests, bench lines
# wide / config / distributed tests, bench lines
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5w
timeout -k 10 120 python tools/digest_run.py > gpurun_out/r5w/digest.txt 2>&1 || { cat gpurun_out/r5w/digest.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r5w/digest.txt

timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_eig.py tests/test_gpu_wide.py tests/test_gpu_bench_pin.py > gpurun_out/r5w/tests.log 2>&1 || { tail -30 gpurun_out/r5w/tests.log; exit 1; }
tail -2 gpurun_out/r5w/tests.log
CFGS="c5 c4 c3" STEPS=10 tools/ab_round.sh r5w ""
