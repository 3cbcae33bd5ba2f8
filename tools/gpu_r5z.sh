#!/bin/bash
# round 5: inverse iteration with a unpredicated 4-set ring + phase-2 spill fix -- bit-identity, eig tests, C5 / C4 kernel sequences
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5z
timeout -k 10 120 python tools/digest_run.py > gpurun_out/r5z/digest.txt 2>&1 || { cat gpurun_out/r5z/digest.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r5z/digest.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_eig.py > gpurun_out/r5z/tests.log 2>&1 || { tail -30 gpurun_out/r5z/tests.log; exit 1; }
tail -2 gpurun_out/r5z/tests.log
for c in c5 c4 c3; do
  RSVD_COOP=0 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r5z/$c -o run -- python3 bench.py --config $c --steps 3 --warmup 1 --cpu-budget 0 > gpurun_out/r5z/$c.log 2>&1 || { echo "rocprof $c failed"; tail -5 gpurun_out/r5z/$c.log; exit 1; }
  f=$(find gpurun_out/r5z/$c -name "*.db" | head -1)
  python3 tools/rocpd_seq.py "$f" > gpurun_out/r5z/${c}_seq.txt && rm -f "$f"
  grep -E "invit|tridiag_kernel|tridiag_bisect" gpurun_out/r5z/${c}_seq.txt; tail -1 gpurun_out/r5z/${c}_seq.txt
done
