#!/bin/bash
# round 5: panel_split at 3 waves / SIMD (launch bounds; 10 VGPR spills) against 2, and the LP = 128 Gram
# chunk cap (2 workgroups per CU) in the C3 bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5v
CFGS="c3" STEPS=20 tools/ab_round.sh r5v "RSVD_GRAM_CAP128=256" "RSVD_GRAM_CAP128=512" "RSVD_GRAM_CAP128=768" "RSVD_GRAM_CAP128=256" "RSVD_GRAM_CAP128=512"
