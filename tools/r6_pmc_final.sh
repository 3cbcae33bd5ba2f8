#!/bin/bash
# Closing PMC passes at the final HEAD: FETCH_SIZE, WRITE_SIZE and the MFMA-busy pass per config, each in
# its own rocprofv3 run (separate --pmc passes, MI355X_MICROARCH.md).  Usage: tools/r6_pmc_final.sh <tag> "<cfgs>"
set -o pipefail
tag=${1:-r06_final4}; cfgs=${2:-"c4 c5 c3"}
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for c in $cfgs; do
  out=$R/gpurun_out/pmc_${tag}_$c
  mkdir -p $out
  B="python3 $R/bench.py --config $c --steps 1 --warmup 1 --cpu-budget 0"
  (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/fetch -o run -- $B > $out/fetch.log 2>&1) || { echo "$c fetch failed"; tail -5 $out/fetch.log; exit 1; }
  (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/write -o run -- $B > $out/write.log 2>&1) || { echo "$c write failed"; tail -5 $out/write.log; exit 1; }
  (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --output-format csv -d $out/mfma -o run -- $B > $out/mfma.log 2>&1) || { echo "$c mfma failed"; tail -5 $out/mfma.log; exit 1; }
  echo "$c passes done"
done
