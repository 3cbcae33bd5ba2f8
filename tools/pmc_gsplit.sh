#!/bin/bash
# PMC passes over tools/wide_lab gsplit (the split Gram at LP = 128 / 256 / 512): stall breakdown and LDS.
set -o pipefail
out=$GRAFT_REPO_ROOT/gpurun_out/pmc_gsplit${1:-}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $out/p1 -o run -- $GRAFT_REPO_ROOT/tools/wide_lab gsplit > $out/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM SQ_INSTS_MFMA --output-format csv -d $out/p2 -o run -- $GRAFT_REPO_ROOT/tools/wide_lab gsplit > $out/p2.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d $out/p3 -o run -- $GRAFT_REPO_ROOT/tools/wide_lab gsplit > $out/p3.log 2>&1 || true
echo ok
