#!/bin/bash
# Benchmark every BASELINE config on one GPU (c2 default line + c3/c4/c5), JSON lines under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
cfgs=${CFGS:-"c2 c3 c4 c5"}
for c in $cfgs; do
  timeout -k 10 300 python -u bench.py --config $c --steps ${STEPS:-10} --warmup ${WARMUP:-3} --cpu-budget ${CPUB:-8} > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || { echo "bench $c failed"; tail -20 gpurun_out/bench_$c.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/bench_$c.json')); r=d['roofline']; c=d['cpu_baseline'] or {}; print('$c', round(d['ms_per_step'],3),'ms', round(d['value'],2), d['unit'], 'roof', r['bound'], round(r['achieved'],1), r['unit'], round(r['frac'],3), 'kernel_us', round(r['avg_launch_us'],1), 'cpu', c.get('value'), d['engine_info'])"
done
