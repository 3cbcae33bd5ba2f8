#!/bin/bash
# round 6 baseline on a fresh box: digests, the whole -m gpu suite, bench lines c4 c5 c3 c2.
# Usage: tools/r6_base.sh <tag>
set -o pipefail
tag=${1:-r6a}
export TMPDIR=/tmp
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 180 python tools/digest_run.py > $out/digest.txt 2>&1 || { cat $out/digest.txt; exit 1; }
grep -v amdgpu.ids $out/digest.txt
if [ -z "$NOTESTS" ]; then
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -2 $out/tests.log
fi
for c in ${CFGS:-c4 c5 c3 c2}; do
  timeout -k 10 200 python -u bench.py --config $c --steps ${STEPS:-20} --warmup 5 --cpu-budget 0 > $out/bench_$c.json 2> $out/bench_$c.err || { echo "bench $c failed"; tail -20 $out/bench_$c.err; exit 1; }
  python -c "import json; d=json.load(open('$out/bench_$c.json')); r=d['roofline']; print('$c', round(d['ms_per_step'],3),'ms', round(r['avg_launch_us'],1), 'us', r.get('frac'))"
done
for c in ${EMU:-}; do  # per-rank kernels of the 8-GPU step (bench.py --emulate-world 8)
  timeout -k 10 200 python -u bench.py --config $c --emulate-world 8 --steps ${STEPS:-20} --warmup 5 --cpu-budget 0 > $out/emu8_$c.json 2> $out/emu8_$c.err || { echo "emu $c failed"; tail -20 $out/emu8_$c.err; exit 1; }
  python -c "import json; d=json.load(open('$out/emu8_$c.json')); print('emu8 $c', round(d['ms_per_step'],3),'ms', d['config']['parallelism'])"
done
