#!/bin/bash
# round 5: twin pacing for the C5 TN halves -- digests, bench A/B, FETCH pass with pacing on
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6h
timeout -k 10 120 python tools/digest_run.py > gpurun_out/r6h/digest.txt 2>&1 || { cat gpurun_out/r6h/digest.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r6h/digest.txt
CFGS="c5" STEPS=10 tools/ab_round.sh r6h "" "RSVD_TWIN_PACE=0" "" "RSVD_TWIN_PACE=0" || exit 1
out=$R/gpurun_out/prof_r6h_c5
mkdir -p $out
(cd /tmp && RSVD_COOP=0 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/fetch -o run -- python3 $R/bench.py --config c5 --steps 3 --warmup 1 --cpu-budget 0 > $out/fetch.log 2>&1) || { tail -5 $out/fetch.log; exit 1; }
python3 - $out/fetch/run_counter_collection.csv <<'PY'
import csv, sys, collections
d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"]
    if "wproj" in k: d[k.split("(")[0][-40:]].append(float(r["Counter_Value"]))
for k, v in d.items(): print(k, len(v), round(2 * sum(v) / len(v) * 1024 / 1e9, 3), "GB")
PY
