#!/bin/bash
# GPU session: the wide / config / full-size GPU tests, then bench A/B lines (env knobs) for c4, c5, c3.
# Usage: tools/ab_round.sh <tag> ["knob settings" ...]   e.g. tools/ab_round.sh v1 "RSVD_GRAM_SPLIT=0" ""
set -o pipefail
tag=${1:-x}; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest -x -v -m gpu --timeout 120 --timeout-method thread $TESTS > gpurun_out/tests_$tag.log 2>&1
  rc=$?; tail -3 gpurun_out/tests_$tag.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" gpurun_out/tests_$tag.log | head -20; exit 1; }
fi
for c in ${CFGS:-c4 c5 c3}; do
  for knobs in "$@"; do
    name=$(echo "$c $knobs" | tr ' =' '__')
    env $knobs timeout -k 10 200 python -u bench.py --config $c --steps ${STEPS:-10} --warmup 3 --cpu-budget 0 > gpurun_out/ab_${tag}_$name.json 2> gpurun_out/ab_${tag}_$name.err || { echo "bench $name failed"; tail -20 gpurun_out/ab_${tag}_$name.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab_${tag}_$name.json')); r=d['roofline']; print('$name', round(d['ms_per_step'],3),'ms', round(r['avg_launch_us'],1), 'us', r.get('sketch',{}).get('avg_launch_us'), d['engine_info']['jacobi_sweeps'], d['check']['ok'])"
  done
done
