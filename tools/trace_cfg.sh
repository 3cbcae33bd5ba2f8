#!/bin/bash
# Kernel-trace stats of one bench config on the default (cooperative) path; the process exits 139
# after the trace is written (rocprofv3 7.2 at exit after a cooperative launch), so this is the last
# GPU step of its call.  Usage: tools/trace_cfg.sh <tag> <config>
set -o pipefail
tag=$1; c=$2
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/prof_${tag}_$c
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 $R/bench.py --config $c --steps 3 --warmup 1 --cpu-budget 0 > $out/trace.log 2>&1
echo "kernel-trace ($c, cooperative launches) rc=$? (139 = the known exit-time fault after the trace is written)"
ls $out/trace
