#!/bin/bash
# rocprofv3 kernel stats of one bench config (no CPU baseline): tools/prof_cfg.sh c4 [steps]
set -o pipefail
export TMPDIR=/tmp
c=${1:-c2}; st=${2:-3}
mkdir -p gpurun_out/prof_$c
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$c -o run -- python3 bench.py --config $c --steps $st --warmup 1 --cpu-budget 0 > gpurun_out/prof_$c.log 2>&1 || { tail -20 gpurun_out/prof_$c.log; exit 1; }
f=$(find gpurun_out/prof_$c -name "*.db" | head -1)
python3 tools/rocpd_stats.py "$f" > gpurun_out/prof_$c.txt && head -20 gpurun_out/prof_$c.txt
