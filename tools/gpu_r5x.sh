#!/bin/bash
# round 5: same-box A/B of the tridiagonalisation's dead-slot skip (RSVD_TRI_NOSKIP=1: the old updates)
set -o pipefail
export TMPDIR=/tmp
CFGS="c5 c4 c3" STEPS=10 tools/ab_round.sh r5x "RSVD_TRI_NOSKIP=1" "" "RSVD_TRI_NOSKIP=1" ""
