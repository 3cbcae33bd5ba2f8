#!/bin/bash
# A/B of the caller's column pitch (bench.py --lda-pad): lda = m against m + pad, alternating on one box.
# Usage: tools/r6_ldapad.sh <tag> "<configs>" "<pads>"
set -o pipefail
tag=${1:-ldapad}; cfgs=${2:-"c3 c4 c5"}; pads=${3:-"0 64 0 64"}
export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
for c in $cfgs; do
  i=0
  for p in $pads; do
    i=$((i+1))
    timeout -k 10 200 python -u bench.py --config $c --steps 10 --warmup 3 --cpu-budget 0 --lda-pad $p > $out/${c}_p${p}_$i.json 2> $out/${c}_p${p}_$i.err || { echo "bench $c pad $p failed"; tail -20 $out/${c}_p${p}_$i.err; exit 1; }
    python -c "import json; d=json.load(open('$out/${c}_p${p}_$i.json')); r=d['roofline']; print('$c pad $p', d['config']['lda'], round(d['ms_per_step'],3), 'ms', round(r['avg_launch_us'],1), 'us', r.get('kernel'), d['check']['ok'])"
  done
done
