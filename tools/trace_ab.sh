#!/bin/bash
# rocprofv3 kernel traces of one config under env knob settings (plain launches: RSVD_COOP=0, see
# common.hpp).  Usage: tools/trace_ab.sh <tag> <config> "KNOB=.. KNOB=.." ...
set -o pipefail
tag=$1; cfg=$2; shift 2
export TMPDIR=/tmp RSVD_COOP=0
mkdir -p gpurun_out
i=0
for knobs in "$@"; do
  out=gpurun_out/trace_${tag}_$i
  env $knobs timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run -- python3 bench.py --cpu-budget 0 --config $cfg --steps 3 --warmup 1 > $out.log 2>&1 || { tail -5 $out.log; exit 1; }
  echo "$i: $knobs" >> gpurun_out/trace_${tag}.idx
  i=$((i+1))
done
