#!/bin/bash
# Exit-time fault under rocprofv3: one kernel-trace pass of the C4 bench with
# the cooperative launches (no RSVD_COOP=0) and the process's /proc/self/maps written just before
# exit, so any fault PCs rocprofv3's handler prints can be mapped to their libraries.  Run LAST in a
# gpurun call (a fault ends the call's GPU work).   Usage: tools/segv_probe.sh <tag>
set -o pipefail
tag=${1:-r04}
out=gpurun_out/segv_$tag
mkdir -p $out
export TMPDIR=/tmp
RSVD_MAPS_OUT=$out/maps.txt timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run \
  -- python3 bench.py --cpu-budget 0 --config c4 --steps 3 --warmup 1 > $out/trace.log 2>&1
rc=$?
echo "rocprofv3 rc=$rc" | tee -a $out/trace.log
exit $rc
