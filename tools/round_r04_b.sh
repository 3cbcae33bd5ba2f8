#!/bin/bash
# Round-4 evidence, part B: per-config PMC passes (FETCH_SIZE, WRITE_SIZE, MFMA busy) with plain
# launches of the persistent kernels (RSVD_COOP=0: clean exits), then the kernel-trace stats of one
# config on the DEFAULT cooperative path LAST -- rocprofv3 7.2 segfaults at the exit of any process
# that made a cooperative launch, after writing the trace (profiles/r04_exit_segv/README.md).
# Usage: tools/round_r04_b.sh <tag> <trace-config> [pmc configs...]
set -o pipefail
tag=${1:-r04}; tc=${2:-c4}; shift 2
cfgs=${@:-c4 c5 c3}
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for c in $cfgs; do
  out=$R/gpurun_out/prof_${tag}_$c
  mkdir -p $out
  (cd /tmp && RSVD_COOP=0 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/fetch -o run -- python3 $R/bench.py --config $c --steps 3 --warmup 1 --cpu-budget 0 > $out/fetch.log 2>&1) || { tail -5 $out/fetch.log; exit 1; }
  (cd /tmp && RSVD_COOP=0 timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/write -o run -- python3 $R/bench.py --config $c --steps 3 --warmup 1 --cpu-budget 0 > $out/write.log 2>&1) || { tail -5 $out/write.log; exit 1; }
  (cd /tmp && RSVD_COOP=0 timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --output-format csv -d $out/mfma -o run -- python3 $R/bench.py --config $c --steps 1 --warmup 1 --cpu-budget 0 > $out/mfma.log 2>&1) || { tail -5 $out/mfma.log; exit 1; }
done
out=$R/gpurun_out/prof_${tag}_$tc
mkdir -p $out
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 $R/bench.py --config $tc --steps 3 --warmup 1 --cpu-budget 0 > $out/trace.log 2>&1
echo "kernel-trace ($tc, cooperative launches) rc=$? (139 = the known exit-time fault after the trace is written)"
ls $out/trace
