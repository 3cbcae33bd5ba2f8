#!/bin/bash
# round 5, call d: staggered TN (RSVD_PROJ_V4=2) bit-identity and A/B at C4
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5d
for v in 0 2; do
  RSVD_PROJ_V4=$v timeout -k 10 120 python tools/digest_run.py > gpurun_out/r5d/digest_v4_$v.txt 2>&1 || { cat gpurun_out/r5d/digest_v4_$v.txt; exit 1; }
  echo "v4=$v"; grep -v amdgpu.ids gpurun_out/r5d/digest_v4_$v.txt
done
CFGS="c4" STEPS=10 tools/ab_round.sh r5d "RSVD_PROJ_V4=0" "RSVD_PROJ_V4=2" "RSVD_PROJ_V4=0" "RSVD_PROJ_V4=2"
