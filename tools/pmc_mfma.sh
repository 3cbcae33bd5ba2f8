#!/bin/bash
# One rocprofv3 PMC pass for MFMA pipe occupancy of a bench config:
#   tools/pmc_mfma.sh c4  -> gpurun_out/pmc_mfma_c4/run_counter_collection.csv
set -o pipefail
c=${1:-c4}
out=$GRAFT_REPO_ROOT/gpurun_out/pmc_mfma_$c
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --output-format csv -d $out -o run \
  -- python3 $GRAFT_REPO_ROOT/bench.py --config $c --steps 1 --warmup 1 --cpu-budget 0 > $out.log 2>&1
