#!/bin/bash
# round 5, call b: the 16x16 diagonal-factor lab (v2 vs DPP), the whole -m gpu suite, A/B bench lines
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5b
timeout -k 10 180 ./tools/wide_lab_cprof chol > gpurun_out/r5b/chol.txt 2>&1 || { cat gpurun_out/r5b/chol.txt; exit 1; }
cat gpurun_out/r5b/chol.txt
timeout -k 10 1500 python -u -m pytest -v -m gpu --timeout 300 --timeout-method thread tests > gpurun_out/r5b/tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/r5b/tests.log | tail -15
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
CFGS="c4 c5 c3" STEPS=10 tools/ab_round.sh r5b "RSVD_CHOL_DIAG=dpp" "RSVD_CHOL_DIAG=v2"
