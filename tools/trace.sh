#!/bin/bash
# rocprofv3 kernel-trace stats of a short bench run: tools/trace.sh <tag> [bench args]
set -o pipefail
tag=$1; shift
out=gpurun_out/trace_$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run -- python3 bench.py --cpu-budget 0 "$@" > $out/trace.log 2>&1 || { tail -20 $out/trace.log; exit 1; }
python3 tools/kstats.py $out/run_kernel_stats.csv 1
