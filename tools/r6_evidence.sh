#!/bin/bash
# round 6 final evidence: bench lines C1-C5 (+ the emulated per-rank C4 / C5 lines), kernel traces of
# C3 / C4 / C5 and of the emulated ranks, the Power l = 2048 timing, then the C4 stall passes.
# Usage: tools/r6_evidence.sh <tag>
set -o pipefail
tag=${1:-r06_final}
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/$tag
mkdir -p $out
for c in c4 c5 c3 c2 c1; do
  timeout -k 10 240 python -u bench.py --config $c --steps 20 --warmup 5 > $out/bench_$c.json 2> $out/bench_$c.err || { echo "bench $c failed"; tail -20 $out/bench_$c.err; exit 1; }
  python -c "import json; d=json.load(open('$out/bench_$c.json')); print('$c', round(d['ms_per_step'],3), 'ms', d['roofline'].get('frac'))"
done
for c in c4 c5; do
  timeout -k 10 200 python -u bench.py --config $c --emulate-world 8 --steps 20 --warmup 5 --cpu-budget 0 > $out/emu8_$c.json 2> $out/emu8_$c.err || { echo "emu $c failed"; exit 1; }
  python -c "import json; d=json.load(open('$out/emu8_$c.json')); print('emu8 $c', round(d['ms_per_step'],3), 'ms')"
done
timeout -k 10 300 python -u -m pytest -q -s -m gpu --timeout 280 --timeout-method thread "tests/test_gpu_big_l.py::test_big_l_power_2048_known_answer" > $out/power2048.log 2>&1 || { tail -20 $out/power2048.log; exit 1; }
grep "Power rSVD" $out/power2048.log
tools/r6_trace.sh $tag "c3 c4 c5" "" || exit 1
BENCH_EXTRA="--emulate-world 8" tools/r6_trace.sh ${tag}_emu8 "c4 c5" "" || exit 1
tools/r6_stall.sh $tag c4
