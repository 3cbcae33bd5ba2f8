#!/bin/bash
# round 5: panel_split In prefetch ring depth -- digests per depth, bench A/B (C3, C5, C4)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6k
for pd in 2 3 4; do
  RSVD_PANEL_PD=$pd timeout -k 10 120 python tools/digest_run.py > gpurun_out/r6k/digest$pd.txt 2>&1 || { cat gpurun_out/r6k/digest$pd.txt; exit 1; }
  echo "PD=$pd"; grep -v amdgpu.ids gpurun_out/r6k/digest$pd.txt
done
CFGS="c3 c5 c4" STEPS=10 tools/ab_round.sh r6k "RSVD_PANEL_PD=2" "RSVD_PANEL_PD=3" "RSVD_PANEL_PD=4" "RSVD_PANEL_PD=2"
