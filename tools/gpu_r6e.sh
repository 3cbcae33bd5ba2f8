#!/bin/bash
# round 5: tridiagonalisation phase-1 hand-off on data-tagged WY apply with whole Y blocks in registers -- lab, bit-identity, eig tests, bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6e
timeout -k 10 60 tools/eig_lab 512 512 4 > gpurun_out/r6e/eiglab.txt 2>&1 && timeout -k 10 60 tools/eig_lab 256 256 4 >> gpurun_out/r6e/eiglab.txt 2>&1 || { cat gpurun_out/r6e/eiglab.txt; exit 1; }
cat gpurun_out/r6e/eiglab.txt
timeout -k 10 120 python tools/digest_run.py > gpurun_out/r6e/digest.txt 2>&1 || { cat gpurun_out/r6e/digest.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r6e/digest.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_eig.py > gpurun_out/r6e/tests.log 2>&1 || { tail -30 gpurun_out/r6e/tests.log; exit 1; }
tail -2 gpurun_out/r6e/tests.log
CFGS="c5 c4 c3" STEPS=10 tools/ab_round.sh r6e ""
