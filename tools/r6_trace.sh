#!/bin/bash
# round 6: kernel traces (rocprofv3 --kernel-trace --stats, plain launches) of configs under env settings.
# Usage: tools/r6_trace.sh <tag> "<cfgs>" "<env A>" "<env B>" ...
set -o pipefail
tag=$1; cfgs=$2; shift 2
export TMPDIR=/tmp RSVD_COOP=0
R=$GRAFT_REPO_ROOT
for c in $cfgs; do
  i=0
  for knobs in "$@"; do
    out=$R/gpurun_out/trace_${tag}_${c}_$i
    mkdir -p $out
    (cd /tmp && env $knobs timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run -- python3 $R/bench.py --cpu-budget 0 --config $c --steps 3 --warmup 1 ${BENCH_EXTRA:-} > $out.log 2>&1) || { tail -5 $out.log; exit 1; }
    echo "$c $i: $knobs" >> $R/gpurun_out/trace_${tag}.idx
    i=$((i+1))
  done
done
