#!/bin/bash
# round 5: SVDMethod::Power past l = 512 (dense_big.cpp + launch_power_grid_rsvd) and the Power / dense tests
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5s
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_big_l.py::test_big_l_power_matches_oracle tests/test_gpu_power.py tests/test_gpu_dense.py > gpurun_out/r5s/tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r5s/tests.log | tail -40; exit $rc
