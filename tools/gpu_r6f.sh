#!/bin/bash
# round 5: C5 / C4 kernel sequences after the WY apply change (RSVD_COOP=0 trace)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6f
for c in c5 c4; do
  RSVD_COOP=0 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r6f/$c -o run -- python3 bench.py --config $c --steps 3 --warmup 1 --cpu-budget 0 > gpurun_out/r6f/$c.log 2>&1 || { echo "rocprof $c failed"; tail -5 gpurun_out/r6f/$c.log; exit 1; }
  f=$(find gpurun_out/r6f/$c -name "*.db" | head -1)
  python3 tools/rocpd_seq.py "$f" > gpurun_out/r6f/${c}_seq.txt && rm -f "$f"
  grep -E "wy_|invit|tridiag|cluster|sqgemm|wproj" gpurun_out/r6f/${c}_seq.txt; tail -1 gpurun_out/r6f/${c}_seq.txt
done
