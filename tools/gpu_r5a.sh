#!/bin/bash
# round 5, call a: the new limit / partition / eigensolver tests, then the gram_reduce A/B bench lines
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5a
timeout -k 10 900 python -u -m pytest -v -m gpu --timeout 300 --timeout-method thread \
  tests/test_gpu_eig.py tests/test_gpu_big_l.py "tests/test_gpu_distributed.py::test_row_sharded_world8_matches_oracle" \
  > gpurun_out/r5a/tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r5a/tests.log | tail -30
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
CFGS="c4 c5 c3" STEPS=10 tools/ab_round.sh r5a "RSVD_GRAM_REDUCE4=0" "RSVD_GRAM_REDUCE4=1"
