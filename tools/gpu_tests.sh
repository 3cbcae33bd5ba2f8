#!/bin/bash
# GPU test pass: pytest -m gpu (one process), log under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ $# -eq 0 ]; then set -- tests; fi
timeout -k 10 600 python -u -m pytest ${PYTEST_X--x} -v -m gpu --timeout 120 --timeout-method thread "$@" > gpurun_out/gpu_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/gpu_tests.log | tail -40
exit $rc
