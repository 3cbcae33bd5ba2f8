#!/bin/bash
# round 5: re-check the A/B knobs' defaults at HEAD (same box, bench lines only)
set -o pipefail
export TMPDIR=/tmp
CFGS="c5" STEPS=10 tools/ab_round.sh r6l "" "RSVD_CHOL2=1" "RSVD_CHOL2=0" "RSVD_PANEL_SPLIT_SHAPE=2" "RSVD_GSPLIT4=0" "" || exit 1
CFGS="c4" STEPS=10 tools/ab_round.sh r6l "" "RSVD_CHOL2=1" "RSVD_CHOL2=0" "RSVD_PANEL_SPLIT_SHAPE=2" "RSVD_PANEL_PD=3" "" || exit 1
CFGS="c3" STEPS=10 tools/ab_round.sh r6l "" "RSVD_TN128=2" "RSVD_GSPLIT_LG=2" "RSVD_PANEL_SPLIT_SHAPE=2" ""
