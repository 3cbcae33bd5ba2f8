#!/bin/bash
# GPU sanity pass: parity tests, smoke, bench, rocprof kernel stats.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 200 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { cat gpurun_out/bench.err | tail; exit 1; }
cat gpurun_out/bench.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --cpu-budget 0 > gpurun_out/prof.log 2>&1 || { tail gpurun_out/prof.log; exit 1; }
find gpurun_out/prof -name '*kernel_stats.csv'
