#!/bin/bash
# round 6 closing evidence: smoke(), the emulated rank 0 of 8 (C4 / C5) and the C4 / C5 kernel traces at
# the final HEAD (plain launches).  Usage: tools/r6_final_c.sh <tag>
set -o pipefail
tag=${1:-r06_final4}
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/$tag
mkdir -p $out
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.txt 2>&1 || { tail -20 $out/smoke.txt; exit 1; }
tail -2 $out/smoke.txt
for c in c4 c5; do
  timeout -k 10 200 python -u bench.py --config $c --emulate-world 8 --steps 20 --warmup 5 --cpu-budget 0 > $out/emu8_$c.json 2> $out/emu8_$c.err || { echo "emu $c failed"; tail -5 $out/emu8_$c.err; exit 1; }
  python -c "import json; d=json.load(open('$out/emu8_$c.json')); print('emu8 $c', round(d['ms_per_step'],3), 'ms')"
done
tools/r6_trace.sh $tag "c4 c5" "" || exit 1
echo traces done
