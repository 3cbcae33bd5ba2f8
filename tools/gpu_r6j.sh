#!/bin/bash
# round 5: branch-free invit multipliers -- digests, eig tests, lab, C5 / C4 sequences
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6j
timeout -k 10 120 python tools/digest_run.py > gpurun_out/r6j/digest.txt 2>&1 || { cat gpurun_out/r6j/digest.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r6j/digest.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_eig.py > gpurun_out/r6j/tests.log 2>&1 || { tail -30 gpurun_out/r6j/tests.log; exit 1; }
tail -2 gpurun_out/r6j/tests.log
timeout -k 10 60 tools/eig_lab 512 512 3 > gpurun_out/r6j/eiglab.txt 2>&1 && timeout -k 10 60 tools/eig_lab 256 256 3 >> gpurun_out/r6j/eiglab.txt 2>&1 || { cat gpurun_out/r6j/eiglab.txt; exit 1; }
grep -E "rep|inverse" gpurun_out/r6j/eiglab.txt
for c in c5 c4; do
  RSVD_COOP=0 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r6j/$c -o run -- python3 bench.py --config $c --steps 3 --warmup 1 --cpu-budget 0 > gpurun_out/r6j/$c.log 2>&1 || { echo "rocprof $c failed"; tail -5 gpurun_out/r6j/$c.log; exit 1; }
  f=$(find gpurun_out/r6j/$c -name "*.db" | head -1)
  python3 tools/rocpd_seq.py "$f" > gpurun_out/r6j/${c}_seq.txt && rm -f "$f"
  grep -E "wy_|invit" gpurun_out/r6j/${c}_seq.txt; tail -1 gpurun_out/r6j/${c}_seq.txt
done
