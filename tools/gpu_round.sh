#!/bin/bash
# One GPU session: the -m gpu suite, the default bench line (C4), its rocprofv3 kernel stats, and
# the FETCH_SIZE calibration pass.  Every step has its own time limit; the first failure ends it.
# Usage: tools/gpu_round.sh <tag> [tests|notests]
set -o pipefail
tag=${1:-x}; mode=${2:-tests}
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "$mode" = tests ]; then
  tools/gpu_tests.sh ${TESTS:-tests} || exit 1
fi
timeout -k 10 300 python3 bench.py > gpurun_out/bench_${tag}.json 2> gpurun_out/bench_${tag}.err || { tail -20 gpurun_out/bench_${tag}.err; exit 1; }
cat gpurun_out/bench_${tag}.json
tools/prof_cfg.sh c4 3 || exit 1
cp gpurun_out/prof_c4.txt gpurun_out/prof_c4_${tag}.txt
if [ -x tools/fetch_calib ]; then
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/calib -o run -- ./tools/fetch_calib > gpurun_out/calib.log 2>&1 || { tail -20 gpurun_out/calib.log; exit 1; }
  cat gpurun_out/calib.log
fi
