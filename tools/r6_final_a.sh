#!/bin/bash
# round 6 final evidence, part A: the -m gpu suite, then the bench lines C1-C5 (default flags: the
# driver's command, CPU baseline included).  Usage: tools/r6_final_a.sh <tag>
set -o pipefail
tag=${1:-r06_final}
export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
timeout -k 10 600 python -u -m pytest -q -m gpu --timeout 200 --timeout-method thread tests > $out/gpu_tests.txt 2>&1 || { tail -40 $out/gpu_tests.txt; exit 1; }
tail -2 $out/gpu_tests.txt
for c in c4 c5 c3 c2 c1; do
  timeout -k 10 240 python -u bench.py --config $c --steps 20 --warmup 5 > $out/bench_$c.json 2> $out/bench_$c.err || { echo "bench $c failed"; tail -20 $out/bench_$c.err; exit 1; }
  python -c "import json; d=json.load(open('$out/bench_$c.json')); print('$c', round(d['ms_per_step'],3), 'ms', d['roofline'].get('frac'))"
done
