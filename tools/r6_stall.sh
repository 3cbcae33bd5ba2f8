#!/bin/bash
# round 6: stall / LDS / cache counter passes of one config's kernels (the C4
# projections' limiter).  Separate rocprofv3 --pmc runs (one block budget each), plain launches.
# Usage: tools/r6_stall.sh <tag> <config>
set -o pipefail
tag=$1; c=$2
export TMPDIR=/tmp RSVD_COOP=0
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/stall_${tag}_$c
mkdir -p $out
B="python3 $R/bench.py --config $c --steps 2 --warmup 1 --cpu-budget 0"
cd /tmp
i=0
for ctr in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM SQ_INSTS_MFMA" \
           "TA_BUSY_avr TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum" \
           "SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES"; do
  timeout -s KILL 240 rocprofv3 --pmc $ctr --output-format csv -d $out/p$i -o run -- $B > $out/p$i.log 2>&1 || { echo "pass $i ($ctr) failed"; tail -5 $out/p$i.log; break; }
  i=$((i+1))
done
python3 $R/tools/pmc_summary.py $out > $out/summary.txt 2>&1
grep -A40 "wproj3tn2_kernel<true\|wproj3_kernel<true, 256, true" $out/summary.txt | head -80
