#!/bin/bash
# Round-4 evidence, part A: the bench line of every config (C4 = the driver's default, with its CPU
# baseline) and the whole -m gpu suite.  Each step has its own limit; the first failure ends the call.
set -o pipefail
tag=${1:-r04}
export TMPDIR=/tmp
mkdir -p gpurun_out/$tag
timeout -k 10 300 python -u bench.py > gpurun_out/$tag/bench_c4.json 2> gpurun_out/$tag/bench_c4.err || { tail -20 gpurun_out/$tag/bench_c4.err; exit 1; }
for c in c5 c3 c2 c1; do
  timeout -k 10 300 python -u bench.py --config $c > gpurun_out/$tag/bench_$c.json 2> gpurun_out/$tag/bench_$c.err || { tail -20 gpurun_out/$tag/bench_$c.err; exit 1; }
done
python3 - "$tag" <<'PY'
import json, sys
for c in ("c1", "c2", "c3", "c4", "c5"):
    d = json.load(open(f"gpurun_out/{sys.argv[1]}/bench_{c}.json"))
    print(c, round(d["ms_per_step"], 3), "ms", round(d["value"], 2), d["unit"], d.get("engine_info"), (d.get("check") or {}).get("ok"))
PY
timeout -k 10 1100 python -u -m pytest -q --timeout 600 --timeout-method thread -m gpu tests > gpurun_out/$tag/gpu_tests.txt 2>&1
rc=$?
tail -5 gpurun_out/$tag/gpu_tests.txt
exit $rc
