#!/bin/bash
# round 5: C5 and C4 kernel sequences at HEAD (RSVD_COOP=0: plain launches, clean exit under rocprofv3)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5n
for c in c5 c4; do
  RSVD_COOP=0 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r5n/$c -o run -- python3 bench.py --config $c --steps 3 --warmup 1 --cpu-budget 0 > gpurun_out/r5n/$c.log 2>&1 || { echo "rocprof $c failed"; tail -5 gpurun_out/r5n/$c.log; exit 1; }
  f=$(find gpurun_out/r5n/$c -name "*.db" | head -1)
  python3 tools/rocpd_seq.py "$f" > gpurun_out/r5n/${c}_seq.txt && rm -f "$f"
  tail -1 gpurun_out/r5n/${c}_seq.txt
done
