#!/bin/bash
# The full-size C4 / C5 oracle pins (tests/test_gpu_bench_pin.py, RSVD_FULLSIZE_PINS=1) with a heartbeat
# line every minute (the oracle's fp64 work prints nothing for minutes).  Usage: tools/r6_fullsize_pins.sh <tag>
set -o pipefail
tag=${1:-fullsize}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp RSVD_FULLSIZE_PINS=1
timeout -k 10 1000 python -u -m pytest -v -s -m gpu --timeout 1100 --timeout-method thread --durations=0 \
  "tests/test_gpu_bench_pin.py::test_bench_fullsize_matches_oracle" "tests/test_gpu_bench_pin.py::test_bench_c3_fullsize_matches_oracle" > $out/log.txt 2>&1 &
pid=$!
while kill -0 $pid 2>/dev/null; do sleep 60; echo "alive $(date +%T)"; tail -1 $out/log.txt; done
wait $pid; rc=$?
tail -12 $out/log.txt
exit $rc
