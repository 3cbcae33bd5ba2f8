#!/bin/bash
# round 5: the leaves' R^-1 inside the register-resident factor's launch -- digests, tests, bench A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r7a
timeout -k 10 120 python tools/digest_run.py > gpurun_out/r7a/digest1.txt 2>&1 || { cat gpurun_out/r7a/digest1.txt; exit 1; }
RSVD_CHOL_RINV_FUSED=0 timeout -k 10 120 python tools/digest_run.py > gpurun_out/r7a/digest0.txt 2>&1 || { cat gpurun_out/r7a/digest0.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r7a/digest1.txt; grep -v amdgpu.ids gpurun_out/r7a/digest0.txt
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_wide.py tests/test_gpu_dense.py tests/test_gpu_parity.py tests/test_gpu_bench_pin.py tests/test_gpu_knob_identity.py > gpurun_out/r7a/tests.log 2>&1 || { tail -30 gpurun_out/r7a/tests.log; exit 1; }
tail -2 gpurun_out/r7a/tests.log
CFGS="c5 c4 c3 c2" STEPS=10 tools/ab_round.sh r7a "" "RSVD_CHOL_RINV_FUSED=0" "" "RSVD_CHOL_RINV_FUSED=0"
