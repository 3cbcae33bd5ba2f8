#!/bin/bash
# round 6: -m gpu suite (optional TESTS=...), then same-box A/B bench lines for the env settings given.
# Usage: tools/r6_ab.sh <tag> "<env settings A>" "<env settings B>" ...   (CFGS, STEPS override)
set -o pipefail
tag=${1:-r6x}; shift
export TMPDIR=/tmp
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 180 python tools/digest_run.py > $out/digest.txt 2>&1 || { cat $out/digest.txt; exit 1; }
grep -v amdgpu.ids $out/digest.txt
if [ "${TESTS:-all}" != "none" ]; then
  T=${TESTS:-tests}; [ "$T" = "all" ] && T=tests
  timeout -k 10 700 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread $T > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
  tail -2 $out/tests.log
fi
for c in ${CFGS:-c4 c5 c3}; do
  for knobs in "$@"; do
    name=$(echo "$c $knobs" | tr ' =' '__')
    env $knobs timeout -k 10 200 python -u bench.py --config $c --steps ${STEPS:-20} --warmup 5 --cpu-budget 0 > $out/ab_$name.json 2> $out/ab_$name.err || { echo "bench $name failed"; tail -20 $out/ab_$name.err; exit 1; }
    python -c "import json; d=json.load(open('$out/ab_$name.json')); r=d['roofline']; print('$name', round(d['ms_per_step'],3),'ms', round(r['avg_launch_us'],1), 'us', d['check'])"
  done
done
