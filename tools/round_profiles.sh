#!/bin/bash
# Round-end evidence in one GPU session: the whole -m gpu suite and smoke(), the bench lines of every
# config (c4 = the driver's default line, with its CPU baseline), then rocprofv3 kernel-trace /
# FETCH_SIZE / WRITE_SIZE passes (tools/profile.sh) and the MFMA-busy pass (tools/pmc_mfma.sh) for
# C4 and C5.  Profiling runs use plain launches (RSVD_COOP=0, common.hpp).  Each step has its own
# time limit; the first failure ends the session.   Usage: tools/round_profiles.sh <tag>
set -o pipefail
tag=${1:-r03_v2}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -2 gpurun_out/${tag}_tests.log
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 || { tail -20 gpurun_out/${tag}_smoke.log; exit 1; }
timeout -k 10 300 python -u bench.py > gpurun_out/${tag}_bench_c4.json 2> gpurun_out/${tag}_bench_c4.err || { tail -20 gpurun_out/${tag}_bench_c4.err; exit 1; }
for c in c5 c3 c2 c1; do
  timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 3 > gpurun_out/${tag}_bench_$c.json 2> gpurun_out/${tag}_bench_$c.err || { tail -20 gpurun_out/${tag}_bench_$c.err; exit 1; }
done
export RSVD_COOP=0
tools/profile.sh ${tag}_c4 --config c4 --steps 3 --warmup 1 > /dev/null || exit 1
tools/profile.sh ${tag}_c5 --config c5 --steps 3 --warmup 1 > /dev/null || exit 1
tools/pmc_mfma.sh c4 || exit 1
tools/pmc_mfma.sh c5 || exit 1
echo done
