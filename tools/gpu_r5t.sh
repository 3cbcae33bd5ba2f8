#!/bin/bash
# round 5: R^-1 pieces from the factor kernels + R12 zero rows in the GEMM epilogue -- bit-identity,
# wide / config / distributed tests, bench lines
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5t
timeout -k 10 120 python tools/digest_run.py > gpurun_out/r5t/digest.txt 2>&1 || { cat gpurun_out/r5t/digest.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r5t/digest.txt
diff <(grep -v amdgpu.ids gpurun_out/r5p/digest0.txt) <(grep -v amdgpu.ids gpurun_out/r5t/digest.txt) && echo "digests identical to r5p"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_wide.py tests/test_gpu_configs.py tests/test_gpu_distributed.py > gpurun_out/r5t/tests.log 2>&1 || { tail -30 gpurun_out/r5t/tests.log; exit 1; }
tail -2 gpurun_out/r5t/tests.log
CFGS="c5 c4 c3" STEPS=10 tools/ab_round.sh r5t ""
