#!/bin/bash
# Round-5 evidence: the bench line of every config (C4 = the driver's default, with its CPU baseline),
# the whole -m gpu suite, then the kernel trace of one config on the cooperative path LAST (rocprofv3
# 7.2 segfaults at the exit of a process that made a cooperative launch, after the trace is written).
# Usage: tools/round_r05_a.sh <tag> [trace-config]
set -o pipefail
tag=${1:-r05}; tc=${2:-c5}
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/$tag
cd $R
timeout -k 10 300 python -u bench.py > gpurun_out/$tag/bench_c4.json 2> gpurun_out/$tag/bench_c4.err || { tail -20 gpurun_out/$tag/bench_c4.err; exit 1; }
for c in c5 c3 c2 c1; do
  timeout -k 10 300 python -u bench.py --config $c > gpurun_out/$tag/bench_$c.json 2> gpurun_out/$tag/bench_$c.err || { tail -20 gpurun_out/$tag/bench_$c.err; exit 1; }
done
python3 - "$tag" <<'PY'
import json, sys
for c in ("c1", "c2", "c3", "c4", "c5"):
    d = json.load(open(f"gpurun_out/{sys.argv[1]}/bench_{c}.json"))
    print(c, round(d["ms_per_step"], 3), "ms", round(d["value"], 2), d["unit"], (d.get("check") or {}).get("ok"))
PY
timeout -k 10 1100 python -u -m pytest -q --timeout 600 --timeout-method thread -m gpu tests > gpurun_out/$tag/gpu_tests.txt 2>&1
rc=$?
tail -3 gpurun_out/$tag/gpu_tests.txt
[ $rc -eq 0 ] || exit $rc
out=$R/gpurun_out/prof_${tag}_$tc
mkdir -p $out
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 $R/bench.py --config $tc --steps 3 --warmup 1 --cpu-budget 0 > $out/trace.log 2>&1
echo "kernel-trace ($tc, cooperative launches) rc=$? (139 = the known exit-time fault after the trace is written)"
ls $out/trace
