#!/bin/bash
# round 5: split panel product with 8 waves per workgroup (M chunk shared by 256 rows) -- lab and bench A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5p
for v in 0 3 0 3; do
  RSVD_PANEL_SPLIT_SHAPE=$v timeout -k 10 60 tools/wide_lab psplit > gpurun_out/r5p/psplit_$v.txt 2>&1 || { cat gpurun_out/r5p/psplit_$v.txt; exit 1; }
  echo "shape $v"; cat gpurun_out/r5p/psplit_$v.txt
done
timeout -k 10 120 python tools/digest_run.py > gpurun_out/r5p/digest0.txt 2>&1 || { cat gpurun_out/r5p/digest0.txt; exit 1; }
RSVD_PANEL_SPLIT_SHAPE=3 timeout -k 10 120 python tools/digest_run.py > gpurun_out/r5p/digest3.txt 2>&1 || { cat gpurun_out/r5p/digest3.txt; exit 1; }
diff <(grep -v amdgpu.ids gpurun_out/r5p/digest0.txt) <(grep -v amdgpu.ids gpurun_out/r5p/digest3.txt) && echo "digests identical"
CFGS="c5 c4 c3" STEPS=10 tools/ab_round.sh r5p "RSVD_PANEL_SPLIT_SHAPE=0" "RSVD_PANEL_SPLIT_SHAPE=3" "RSVD_PANEL_SPLIT_SHAPE=0" "RSVD_PANEL_SPLIT_SHAPE=3"
