#!/bin/bash
# round 6 final evidence, part B: the emulated rank-0-of-8 bench lines (C4 / C5), the Power l = 2048
# timing, kernel traces of C3 / C4 / C5 and of the emulated ranks, then the C4 stall passes.
# Usage: tools/r6_final_b.sh <tag>
set -o pipefail
tag=${1:-r06_final}
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/$tag
mkdir -p $out
for c in c4 c5; do
  timeout -k 10 200 python -u bench.py --config $c --emulate-world 8 --steps 20 --warmup 5 --cpu-budget 0 > $out/emu8_$c.json 2> $out/emu8_$c.err || { echo "emu $c failed"; tail -5 $out/emu8_$c.err; exit 1; }
  python -c "import json; d=json.load(open('$out/emu8_$c.json')); print('emu8 $c', round(d['ms_per_step'],3), 'ms')"
done
timeout -k 10 300 python -u -m pytest -q -s -m gpu --timeout 280 --timeout-method thread "tests/test_gpu_big_l.py::test_big_l_power_2048_known_answer" > $out/power2048.log 2>&1 || { tail -20 $out/power2048.log; exit 1; }
grep -i "power" $out/power2048.log | tail -3
tools/r6_trace.sh $tag "c3 c4 c5" "" || exit 1
BENCH_EXTRA="--emulate-world 8" tools/r6_trace.sh ${tag}_emu8 "c4 c5" "" || exit 1
tools/r6_stall.sh $tag c4 > /dev/null && echo "stall passes done"
