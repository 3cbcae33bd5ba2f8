#!/bin/bash
# round 5: SQ counters of gram_pieces_kernel against gram_split4_kernel (tools/wide_lab gpieces)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r5r
mkdir -p $out
cd /tmp
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $out/p1 -o run -- $R/tools/wide_lab gpieces > $out/p1.log 2>&1 || { tail -5 $out/p1.log; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM SQ_INSTS_MFMA --output-format csv -d $out/p2 -o run -- $R/tools/wide_lab gpieces > $out/p2.log 2>&1 || { tail -5 $out/p2.log; exit 1; }
timeout -k 10 60 $R/tools/wide_lab ppieces > $out/ppieces.txt 2>&1 || { cat $out/ppieces.txt; exit 1; }; cat $out/ppieces.txt
python3 $R/tools/pmc_summary.py $out > $out/pmc.txt; grep -A12 "gram_pieces\|gram_split4" $out/pmc.txt | head -80
