#!/bin/bash
# SQ / LDS / cache counters of the C4 projection kernels (wide_lab proj4), one rocprofv3 pass each.
set -o pipefail
mkdir -p gpurun_out/pmc_proj
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/pmc_proj/avail.txt 2>&1 || true
i=0
for set in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc_proj/p$i -o pmc -- ./tools/wide_lab proj4 > gpurun_out/pmc_proj/p$i.log 2>&1 || { tail -5 gpurun_out/pmc_proj/p$i.log; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/pmc_proj
