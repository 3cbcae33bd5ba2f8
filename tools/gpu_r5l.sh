#!/bin/bash
# round 5: C3 A/B of the LP = 128 TN K phases in the engine
set -o pipefail
export TMPDIR=/tmp
CFGS="c3" STEPS=20 tools/ab_round.sh r5l "RSVD_TN128_PHASES=1" "RSVD_TN128_PHASES=8" "RSVD_TN128_PHASES=1" "RSVD_TN128_PHASES=8" "RSVD_TN128_PHASES=16"
