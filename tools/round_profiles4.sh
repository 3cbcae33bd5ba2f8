#!/bin/bash
# Round-4 evidence in one GPU session: bench lines of every config (c4 = the driver's default line,
# with its CPU baseline), then rocprofv3 passes -- kernel-trace stats, FETCH_SIZE / WRITE_SIZE
# (tools/profile.sh) and MFMA busy (tools/pmc_mfma.sh) -- for C4, C5 and C3, all on the default
# (cooperative) launch path.  Each step has its own time limit; the first failure ends the session.
# Usage: tools/round_profiles4.sh <tag> [configs...]
set -o pipefail
tag=${1:-r04}; shift
cfgs=${@:-c4 c5 c3}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py > gpurun_out/${tag}_bench_c4.json 2> gpurun_out/${tag}_bench_c4.err || { tail -20 gpurun_out/${tag}_bench_c4.err; exit 1; }
for c in c5 c3 c2 c1; do
  timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 3 > gpurun_out/${tag}_bench_$c.json 2> gpurun_out/${tag}_bench_$c.err || { tail -20 gpurun_out/${tag}_bench_$c.err; exit 1; }
done
for c in $cfgs; do
  tools/profile.sh ${tag}_$c --config $c --steps 3 --warmup 1 > /dev/null || exit 1
  tools/pmc_mfma.sh $c || exit 1
  mv gpurun_out/pmc_mfma_$c gpurun_out/${tag}_pmc_mfma_$c
done
echo done
