#!/bin/bash
# round 5, call c: diag-factor lab re-check, v4 TN bit-identity (digest) and A/B, Cholesky-path tests
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5c
timeout -k 10 180 ./tools/wide_lab_cprof chol > gpurun_out/r5c/chol.txt 2>&1 || { cat gpurun_out/r5c/chol.txt; exit 1; }
head -3 gpurun_out/r5c/chol.txt
for v in 0 1; do
  RSVD_PROJ_V4=$v timeout -k 10 120 python tools/digest_run.py > gpurun_out/r5c/digest_v4_$v.txt 2>&1 || { cat gpurun_out/r5c/digest_v4_$v.txt; exit 1; }
  echo "v4=$v"; cat gpurun_out/r5c/digest_v4_$v.txt
done
timeout -k 10 900 python -u -m pytest -v -m gpu --timeout 300 --timeout-method thread tests/test_gpu_dense.py tests/test_gpu_wide.py tests/test_gpu_configs.py tests/test_gpu_parity.py > gpurun_out/r5c/tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/r5c/tests.log | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
RSVD_PROJ_V4=1 timeout -k 10 300 python -u -m pytest -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_wide.py tests/test_gpu_bench_pin.py > gpurun_out/r5c/tests_v4.log 2>&1
rc=$?
tail -3 gpurun_out/r5c/tests_v4.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
CFGS="c4" STEPS=10 tools/ab_round.sh r5c "RSVD_PROJ_V4=0" "RSVD_PROJ_V4=1" "RSVD_PROJ_V4=0" "RSVD_PROJ_V4=1"
