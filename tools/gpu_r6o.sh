#!/bin/bash
# round 5: one-workgroup tridiagonalisation split at 128 rows -- eig / wide / pin tests, lab, bench A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6o
timeout -k 10 120 python tools/digest_run.py > gpurun_out/r6o/digest1.txt 2>&1 || { cat gpurun_out/r6o/digest1.txt; exit 1; }
RSVD_TRI_SPLIT2=0 timeout -k 10 120 python tools/digest_run.py > gpurun_out/r6o/digest0.txt 2>&1 || { cat gpurun_out/r6o/digest0.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r6o/digest1.txt; grep -v amdgpu.ids gpurun_out/r6o/digest0.txt
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_eig.py tests/test_gpu_wide.py tests/test_gpu_bench_pin.py tests/test_gpu_knob_identity.py > gpurun_out/r6o/tests.log 2>&1 || { tail -30 gpurun_out/r6o/tests.log; exit 1; }
tail -2 gpurun_out/r6o/tests.log
timeout -k 10 60 tools/eig_lab 512 512 3 > gpurun_out/r6o/eiglab.txt 2>&1 && timeout -k 10 60 tools/eig_lab 256 256 3 >> gpurun_out/r6o/eiglab.txt 2>&1 && timeout -k 10 60 tools/eig_lab 160 256 3 >> gpurun_out/r6o/eiglab.txt 2>&1 || { cat gpurun_out/r6o/eiglab.txt; exit 1; }
grep "rep 2" gpurun_out/r6o/eiglab.txt
CFGS="c5 c4" STEPS=10 tools/ab_round.sh r6o "" "RSVD_TRI_SPLIT2=0" "" "RSVD_TRI_SPLIT2=0"
