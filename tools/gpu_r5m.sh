#!/bin/bash
# round 5: C3 kernel trace at HEAD (cooperative path; run last -- exit SIGSEGV after the trace is written)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5m
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5m/c3 -o run -- python3 bench.py --config c3 --steps 5 --warmup 1 --cpu-budget 0 > gpurun_out/r5m/c3.log 2>&1
rc=$?; echo "rocprof rc $rc"
f=$(find gpurun_out/r5m/c3 -name "*.db" | head -1)
python3 tools/rocpd_stats.py "$f" tridiag_bisect_kernel > gpurun_out/r5m/c3_stats.txt && python3 tools/rocpd_seq.py "$f" > gpurun_out/r5m/c3_seq.txt
cp gpurun_out/r5m/c3/*kernel_stats.csv gpurun_out/r5m/c3_kernel_stats.csv 2>/dev/null || find gpurun_out/r5m/c3 -name "*kernel_stats.csv" -exec cp {} gpurun_out/r5m/c3_kernel_stats.csv \;
rm -f "$f"
head -5 gpurun_out/r5m/c3_stats.txt; tail -3 gpurun_out/r5m/c3_seq.txt
